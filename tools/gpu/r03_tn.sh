#!/bin/bash
# TN split plan (one round), embed affine fin: tests, C3 step, C3 op profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "weight_grad or embedding_grad or embed_ln_bwd" -q --timeout 120 --timeout-method thread > gpurun_out/r03_tn_test.log 2>&1
rc=$?; tail -2 gpurun_out/r03_tn_test.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_tn_test.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 > gpurun_out/r03_c3_tn.log 2>&1 || { tail -20 gpurun_out/r03_c3_tn.log; exit 1; }
tail -1 gpurun_out/r03_c3_tn.log
TRAIN_OUT=r03_trainprof3 bash tools/gpu/trainprof.sh > gpurun_out/r03_trainprof3.txt 2>&1 || exit 1
head -30 gpurun_out/r03_trainprof3.txt
timeout -k 10 300 python tools/train_opprof.py > gpurun_out/r03_opprof.txt 2>&1 || { tail -5 gpurun_out/r03_opprof.txt; exit 1; }
echo opprof ok
