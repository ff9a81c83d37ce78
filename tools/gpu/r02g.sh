#!/bin/bash
# round-2 session g: training GPU tests + C3 A/B of the bf16 global-branch dh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || { tail -30 gpurun_out/pytest_train.log; exit 1; }
tail -n 2 gpurun_out/pytest_train.log
for i in 1 2; do
  timeout -k 10 200 python tools/train_bench.py --steps 20 > gpurun_out/tb_g_new_$i.log 2>&1 || exit 1
  timeout -k 10 200 python tools/train_bench.py --steps 20 --global-dh-f32 > gpurun_out/tb_g_f32_$i.log 2>&1 || exit 1
done
for f in gpurun_out/tb_g_*.log; do echo "$f $(tail -n 1 $f)"; done
