#!/bin/bash
# GEMM epilogue round: GEMM/model GPU tests, the store-policy A/B, a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1
rc=$?; tail -3 gpurun_out/epi_tests.log; [ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/epi_tests.log | head -20; exit 1; }
timeout -k 10 300 python3 tools/gemm_var.py 2>&1 | tee gpurun_out/gemm_var.log || exit 1
