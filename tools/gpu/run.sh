#!/bin/bash
# One parametrised GPU driver (replaces the per-round one-off launchers).
#   bash tools/gpu/run.sh <mode> [tag]      (inside gpurun; outputs under gpurun_out/<tag>/)
# modes:
#   suite      the whole -m gpu suite, then smoke() (the round-end gates)
#   tests      pytest on $TESTS (default: the whole -m gpu suite), then a short bench line
#   bench      the default bench.py line (N=1)
#   profile    tools/profile_bench.sh: rocprofv3 kernel trace + FETCH / WRITE / MFMA-busy passes, then
#              the default bench line from the same build
#   gemm       GEMM shape timings, the four-wave kernels 16x16x32 vs 32x32x16 (knob gemm_mfma32),
#              alternated twice (tools/gemm_var.py)
#   lines      C3 (captured bf16 / fp16+GradScaler+accumulation+clip, eager), C4 (captured, 4 and 32 per
#              rank) and C5 (retrieval, catalog encode) lines plus the retrieval kernel trace
#   torchops   the Python lines that launch torch (non-HIP) kernels in one eager C3 step
#   trainprof  rocprofv3 kernel trace of the captured C3 step ($TRAIN_ARGS)
#   abc3       captured-C3 A/Bs listed in $AB (knob:<name>[=a,b] or a Python flag), $TRAIN_ARGS appended
#   abc2       C2 forward-step A/Bs listed in $AB (tools/ab_step.py arguments)
#   abc5       C5 retrieval, rank_w32 0 / 1 alternated by process
#   abtree     same-box A/B of library generations: abtree/<name> trees (tools/abtree.sh, $TREES, default
#              "r03 r04") against the working tree, every row through the last layer, order A B C C B A
#   gemmpmc    the four C2 GEMMs alone (tools/gemm_pmc.py): kernel trace + SQ wait / instruction / LDS and
#              HBM-byte PMC passes, one rocprofv3 run per pass
#   gemmbar    same-box GEMM bar at the C2 shapes: hipBLASLt plain / bias vs the HIP kernels, legs round-robin
#              in one process, knob variants from $KNOBS (tools/gemm_c2_bar.py)
#   bandab     band attention pipe2 vs pipe3 (knob band_path 0 / 3): kernel traces of C2 steps, ABBA by process
#   c5ab       C5 retrieval, rank kernel families w16 / w32 with the top-k, same results required, plus a
#              kernel trace of the 125k shard (tools/retrieval_bench.py --family, tools/trace_seq.py)
#   ab32       same-process A/B of the 32x32x16 GEMM kernel (knob gemm_mfma32): C2 forward, captured C3;
#              C5 retrieval with the 32x32x16 rank kernel (knob rank_w32) alternated by process
set -o pipefail
MODE=${1:?mode}
TAG=${2:-$MODE}
O=gpurun_out/$TAG
mkdir -p $O
fail() { tail -${2:-30} "$1"; exit 1; }
case $MODE in
  suite)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${SUITE_ARGS:-} \
      > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED" $O/pytest.log | cut -c1-300 | head -20; fail $O/pytest.log 5; }
    tail -2 $O/pytest.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
      || fail $O/smoke.log 5
    tail -1 $O/smoke.log ;;
  tests)
    timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} ${PYTEST_X--x} -v --timeout 300 --timeout-method thread \
      > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED" $O/pytest.log | cut -c1-300 | head -30; fail $O/pytest.log 5; }
    grep -E "passed|failed" $O/pytest.log | tail -1
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > $O/bench.log 2>&1 \
      || fail $O/bench.log 20
    tail -1 $O/bench.log | cut -c1-300 ;;
  bench)
    timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || fail $O/bench.log 20
    tail -1 $O/bench.log | cut -c1-600 ;;
  profile)
    bash tools/profile_bench.sh $TAG > $O/profile.log 2>&1 || fail $O/profile.log
    cat gpurun_out/prof_$TAG/summary.txt
    timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || fail $O/bench.log 20
    tail -1 $O/bench.log | cut -c1-600 ;;
  gemm)
    for rep in 1 2; do
      for k in gemm_mfma32=0 gemm_mfma32=1; do
        RF_KNOBS=$k timeout -k 10 200 python3 tools/gemm_var.py >> $O/gemm.log 2>&1 || fail $O/gemm.log
      done
    done
    cat $O/gemm.log ;;
  ab32)
    # the 32x32x16 four-wave GEMM vs the 16x16x32 one: C2 forward steps and captured C3 steps, each A/B
    # alternated in one process (knob gemm_mfma32)
    AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py knob:gemm_mfma32 64 > $O/ab_c2.log 2>&1 || fail $O/ab_c2.log
    cat $O/ab_c2.log
    AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py knob:gfold_chunk=128,0 64 > $O/ab_c2_gf.log 2>&1 \
      || fail $O/ab_c2_gf.log
    cat $O/ab_c2_gf.log
    # raster: every N-tile of an A row-panel on one XCD (gemm_gn 0 = full width) vs groups of 6, on w32
    RF_KNOBS=gemm_mfma32=1 AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py knob:gemm_gn=0,6 64 \
      > $O/ab_c2_gn.log 2>&1 || fail $O/ab_c2_gn.log
    cat $O/ab_c2_gn.log
    timeout -k 10 500 python tools/train_bench.py --graph --steps 8 --warmup 2 --ab-knob gemm_mfma32 > $O/ab_c3.log 2>&1 \
      || fail $O/ab_c3.log
    tail -2 $O/ab_c3.log
    timeout -k 10 500 python tools/train_bench.py --graph --steps 8 --warmup 2 --ab DW_SIDE_STREAM > $O/ab_c3_side.log 2>&1 \
      || fail $O/ab_c3_side.log
    tail -2 $O/ab_c3_side.log
    for k in rank_w32=0 rank_w32=1 rank_w32=0 rank_w32=1; do
      RF_KNOBS=$k timeout -k 10 300 python tools/retrieval_bench.py >> $O/ab_c5.log 2>&1 || fail $O/ab_c5.log
      echo "$k" >> $O/ab_c5.log
    done
    grep -E "rank_w32|ms" $O/ab_c5.log | cut -c1-250 ;;
  abtree)
    trees="${TREES:-r03 r04} cur"
    order="$trees $(echo $trees | tr ' ' '\n' | tac | tr '\n' ' ')"
    for t in $order; do
      if [ "$t" = cur ]; then dir=.; extra="--full-last-layer --no-full-leg"; else dir=abtree/$t; extra=""; fi
      [ "$t" != cur ] && grep -q full-last-layer $dir/bench.py && extra="--full-last-layer"
      (cd $dir && timeout -k 10 300 python bench.py --steps 80 --warmup 10 --cpu-baseline-seconds 0 $extra) \
        > $O/ab_$t.log 2>&1 || fail $O/ab_$t.log
      tail -1 $O/ab_$t.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
k = d.get('kernels', {})
print(json.dumps({'tree': '$t', 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  **{n: round(k[n]['avg_us'], 1) for n in ('gemm_qkv', 'gemm_out', 'gemm_ffn1', 'gemm_ffn2', 'band_attn')
                     if n in k}}))" | tee -a $O/abtree.jsonl
    done ;;
  gemmpmc)
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o g -- \
      python3 tools/gemm_pmc.py 40 > $O/trace.log 2>&1 || fail $O/trace.log
    i=0
    for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES" \
                "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
      timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $O/pmc$i -o p -- python3 tools/gemm_pmc.py 10 \
        > $O/pmc$i.log 2>&1 || fail $O/pmc$i.log
      i=$((i+1))
    done
    python3 tools/summarize_pmc.py $O | tee $O/summary.txt ;;
  abc3)
    # captured C3 steps, one same-process A/B per entry of $AB: knob:<name>[=a,b] or a Python flag name
    n=0
    for x in ${AB:?AB}; do
      n=$((n + 1))
      case $x in knob:*) arg="--ab-knob ${x#knob:}" ;; *) arg="--ab $x" ;; esac
      timeout -k 10 500 python tools/train_bench.py --graph --steps 8 --warmup 2 ${TRAIN_ARGS:-} $arg \
        > $O/abc3_$n.log 2>&1 || fail $O/abc3_$n.log
      echo "== $x"; tail -2 $O/abc3_$n.log
    done ;;
  abc2)
    # C2 forward steps, one same-process A/B per entry of $AB (knob:<name>[=a,b] or a models / train flag)
    n=0
    for x in ${AB:?AB}; do
      n=$((n + 1))
      AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py $x 64 > $O/abc2_$n.log 2>&1 || fail $O/abc2_$n.log
      echo "== $x"; grep -E "ms/step|diff" $O/abc2_$n.log
    done ;;
  abc5)
    # C5 retrieval with the 32x32x16 rank kernel (knob rank_w32) alternated by process
    for k in rank_w32=0 rank_w32=1 rank_w32=0 rank_w32=1; do
      RF_KNOBS=$k timeout -k 10 300 python tools/retrieval_bench.py >> $O/ab_c5.log 2>&1 || fail $O/ab_c5.log
      echo "$k" >> $O/ab_c5.log
    done
    grep -E "rank_w32|ms" $O/ab_c5.log | cut -c1-250 ;;
  lines)
    for args in "--graph" "--graph --dtype fp16 --accum 2 --clip 1.0" "--graph --negatives 1000" ""; do
      timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 $args > $O/c3.log 2>&1 || fail $O/c3.log 20
      tail -1 $O/c3.log | tee -a $O/c3_lines.jsonl
    done
    for b in 4 32; do
      timeout -k 10 300 python tools/pretrain_bench.py --batch $b --steps 6 --warmup 2 --graph > $O/c4.log 2>&1 \
        || fail $O/c4.log 20
      tail -1 $O/c4.log | tee -a $O/c4_lines.jsonl
    done
    timeout -k 10 300 python tools/retrieval_bench.py > $O/retrieval.log 2>&1 || fail $O/retrieval.log 20
    tail -4 $O/retrieval.log
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/retrieval_trace -o r -- \
      python3 tools/retrieval_bench.py > $O/retrieval_trace.log 2>&1 || fail $O/retrieval_trace.log 20
    timeout -k 10 600 python tools/catalog_bench.py > $O/catalog.log 2>&1 || fail $O/catalog.log 20
    tail -2 $O/catalog.log ;;
  gemmbar)
    timeout -k 10 400 python tools/gemm_c2_bar.py ${KNOBS:-} > $O/bar.jsonl 2>&1 || fail $O/bar.jsonl
    cut -c1-160 $O/bar.jsonl ;;
  bandab)
    for run in 0a 3a 3b 0b; do
      bp=${run:0:1}
      ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && RF_KNOBS=band_path=$bp timeout -k 10 300 \
        rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$run -o c2 -- python3 tools/c2_steps.py 40 10 \
        > $O/run_$run.log 2>&1 ) || fail $O/run_$run.log
      grep ms/step $O/run_$run.log
      python3 tools/summarize_profile.py $O/trace_$run --config 64,1024,12 > $O/summary_$run.txt 2>&1 || true
    done ;;
  c5ab)
    timeout -k 10 400 python tools/retrieval_bench.py --family w16,w32 > $O/retrieval.log 2>&1 || fail $O/retrieval.log
    grep -E '"ms"' $O/retrieval.log | cut -c1-200
    ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace \
      --output-format csv -d $O/trace -o r -- python3 tools/retrieval_bench.py --items 125000 > $O/trace.log 2>&1 ) \
      || fail $O/trace.log
    python3 tools/trace_seq.py $O/trace/r_kernel_trace.csv 0 45 | tail -36 ;;
  torchops)
    timeout -k 10 300 python tools/torch_ops_trace.py > $O/torchops.txt 2>&1 || fail $O/torchops.txt 20
    head -80 $O/torchops.txt ;;
  trainprof)
    TRAIN_OUT=$TAG/trace TRAIN_ARGS=${TRAIN_ARGS:---graph} bash tools/gpu/trainprof.sh > $O/trainprof.txt 2>&1 \
      || fail $O/trainprof.txt 20
    head -30 $O/trainprof.txt ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
