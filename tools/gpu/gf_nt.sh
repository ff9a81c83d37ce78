# A/B of the global-fold partial pass's image stream with the non-temporal policy (tools/varx/librf_gfnt.so,
# tools/build_variant.sh gfnt rf_global.hip -DRF_GF_NT=1) against the product library: isolated kernel times
# under rocprofv3, then the C2 bench in alternating processes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gfnt
mkdir -p $O
for v in prod nt prod2 nt2; do
  lib=""; case $v in nt*) lib=$GRAFT_REPO_ROOT/tools/varx/librf_gfnt.so ;; esac
  RF_HIP_LIB=$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python3 tools/gfold_bench.py > $O/$v.log 2>&1
  echo "== $v"; find $O/$v -name "*kernel_stats.csv" -exec grep -h "partial_bf16" {} \; | cut -d, -f1-7
done
for v in prod nt prod2 nt2; do
  lib=""; case $v in nt*) lib=$GRAFT_REPO_ROOT/tools/varx/librf_gfnt.so ;; esac
  RF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline-seconds 0 --no-full-leg --no-kernel-timing > $O/bench_$v.log 2>&1
  echo "== bench $v: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
