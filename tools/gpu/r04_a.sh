#!/bin/bash
# round-4 check: optimizer / captured-step tests, GEMM kernels (both MFMA shapes), GEMM A/B, short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_graphs.py "tests/test_gpu_kernels.py::test_gemm_four_wave_kernels_all_epilogues" "tests/test_gpu_kernels.py::test_cos_scores_bwd_matches_autograd" tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r04a_pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for k in gemm_mfma32=0 gemm_mfma32=1; do
    RF_KNOBS=$k timeout -k 10 200 python3 tools/gemm_var.py >> gpurun_out/r04a_gemm.log 2>&1 || exit 1
  done
done
cat gpurun_out/r04a_gemm.log
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r04a_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r04a_bench.log | cut -c1-300; exit $rc
