# diagnostic: where the C2 fold partial pass spends its time. Normal build, then RF_GF_DIAG builds of
# rf_global.hip (tools/build_variant.sh gfdiagN rf_global.hip -DRF_GF_DIAG=N, moved to tools/varx):
# 1 no score MFMAs, 2 no refill DMA (stale image), 4 no P.H products, 5 = 1 + 4; and h with a padded
# row stride (RF_GF_PADCOLS). Kernel times from rocprofv3 --kernel-trace --stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gfd
mkdir -p $O
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o k -- python3 tools/gfold_bench.py > $O/base.log 2>&1
RF_GF_PADCOLS=64 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pad64 -o k -- python3 tools/gfold_bench.py > $O/pad64.log 2>&1
RF_KNOBS=gfold_path=4 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ring -o k -- python3 tools/gfold_bench.py > $O/ring.log 2>&1
for d in 1 2 4 5; do
  RF_HIP_LIB=$GRAFT_REPO_ROOT/tools/varx/librf_gfdiag$d.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o k -- python3 tools/gfold_bench.py > $O/d$d.log 2>&1
done
for f in $O/*/; do echo "== $f"; find $f -name "*kernel_stats.csv" -exec grep -i gfold {} \; ; done > $O/summary.txt
cat $O/summary.txt
