#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_all2.log 2>&1
rc=$?; tail -2 gpurun_out/r03_gpu_all2.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_gpu_all2.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_opprof.py > gpurun_out/r03_opprof3.txt 2>&1 || { tail -5 gpurun_out/r03_opprof3.txt; exit 1; }
TRAIN_OUT=r03_trainprof4 TRAIN_ARGS=--graph bash tools/gpu/trainprof.sh > gpurun_out/r03_trainprof4.txt 2>&1 || exit 1
head -30 gpurun_out/r03_trainprof4.txt
