# diagnostic: global fold kernels under rocprofv3 with the normal and RF_GF_DIAG builds
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gf/base -o k -- python3 tools/gfold_bench.py
RF_GFOLD_GEMV=1 timeout -k 10 120 python3 tools/gfold_bench.py
for d in 1 2 4; do
  RF_HIP_LIB=$GRAFT_REPO_ROOT/recformer_amd/csrc/build/libdiag$d.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gf/d$d -o k -- python3 tools/gfold_bench.py
done
