# global-fold partial prologue A/B: parity tests of the fold, the stamps timeline of the new order, and
# kernel times of the product vs the old-order build (tools/varx/librf_gfold.so) under rocprofv3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gfp
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fold or global or catalog" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
RF_HIP_LIB=$GRAFT_REPO_ROOT/tools/varx/librf_gfstamps2.so timeout -k 10 150 python3 tools/gfold_stamps.py > $O/stamps_new.log 2>&1
tail -17 $O/stamps_new.log
for v in prod old prod2 old2; do
  lib=""; case $v in old*) lib=$GRAFT_REPO_ROOT/tools/varx/librf_gfold.so ;; esac
  RF_HIP_LIB=$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python3 tools/gfold_bench.py > $O/$v.log 2>&1
  echo "== $v"; find $O/$v -name "*kernel_stats.csv" -exec grep -i "partial_bf16\|qu_mfma\|out16" {} \; | cut -d, -f1-7
done
# step level: the C2 bench in alternating processes (no CPU leg, no full-last-layer leg)
for v in prod old prod2 old2; do
  lib=""; case $v in old*) lib=$GRAFT_REPO_ROOT/tools/varx/librf_gfold.so ;; esac
  RF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline-seconds 0 --no-full-leg --no-kernel-timing > $O/bench_$v.log 2>&1
  echo "== bench $v: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
