#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_model.py -k "fold or global" -q --timeout 200 --timeout-method thread > gpurun_out/r03_fold2.log 2>&1
rc=$?; tail -2 gpurun_out/r03_fold2.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_fold2.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/ab_knob.py gfold_path 0 1 > gpurun_out/r03_fold_ab.log 2>&1 || { tail -20 gpurun_out/r03_fold_ab.log; exit 1; }
tail -3 gpurun_out/r03_fold_ab.log | cut -c1-600
