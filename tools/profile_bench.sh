#!/bin/bash
# rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes over a short
# bench run; writes gpurun_out/prof_<tag>/ and a per-kernel summary JSON.
set -e
TAG=${1:-r01}
# no batch sweep under the profiler: its replayed HIP graphs crash rocprofv3's PMC passes (SIGSEGV in
# CUDAGraph.replay, gpurun_out/prof_r06f/fetch.log), and the sweep is not the profiled workload
ARGS="--steps ${PROF_STEPS:-30} --warmup 10 --cpu-baseline-seconds 0 --no-kernel-timing --batch-sweep= ${BENCH_ARGS:-}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o bench -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o bench -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/mfma -o bench -- python3 bench.py $ARGS > $OUT/mfma.log 2>&1
python3 tools/summarize_profile.py $OUT ${SUMMARY_ARGS:-} > $OUT/summary.txt
cat $OUT/summary.txt
