#!/bin/bash
# Round 3: LM-head HIP test, C3 step time, C3 kernel trace summary, C4 step times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -k "decoder_ce or lm_head or pretrain" -v --timeout 300 --timeout-method thread > gpurun_out/r03_lmhead.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_lmhead.log | tail -12
[ $rc -eq 0 ] || { grep -E "^E  " gpurun_out/r03_lmhead.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 > gpurun_out/r03_c3.log 2>&1 || { tail -20 gpurun_out/r03_c3.log; exit 1; }
tail -2 gpurun_out/r03_c3.log
TRAIN_OUT=r03_trainprof bash tools/gpu/trainprof.sh || exit 1
timeout -k 10 300 python tools/pretrain_bench.py --batch 4 --steps 6 --warmup 2 > gpurun_out/r03_c4_b4.log 2>&1 || { tail -20 gpurun_out/r03_c4_b4.log; exit 1; }
tail -1 gpurun_out/r03_c4_b4.log
timeout -k 10 300 python tools/pretrain_bench.py --batch 32 --steps 4 --warmup 2 > gpurun_out/r03_c4_b32.log 2>&1 || { tail -20 gpurun_out/r03_c4_b32.log; exit 1; }
tail -1 gpurun_out/r03_c4_b32.log
