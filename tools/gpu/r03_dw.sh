#!/bin/bash
# Round 3: HIP weight-gradient kernel + band pipe3 — parity tests, then same-process A/Bs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "weight_grad or pipe3 or band_and_global" -q --timeout 300 --timeout-method thread > gpurun_out/r03_dw_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_dw_test.log
[ $rc -eq 0 ] || { grep -E "^E  |Error|FAILED" gpurun_out/r03_dw_test.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -k "c2_finetune or full_softmax or pretrain_training" -q --timeout 300 --timeout-method thread > gpurun_out/r03_dw_train.log 2>&1
rc=$?; tail -3 gpurun_out/r03_dw_train.log
[ $rc -eq 0 ] || { grep -E "^E  |Error|FAILED" gpurun_out/r03_dw_train.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/ab_knob.py band_path 0 3 > gpurun_out/r03_ab_band.log 2>&1 || { tail -20 gpurun_out/r03_ab_band.log; exit 1; }
cat gpurun_out/r03_ab_band.log | cut -c1-600
timeout -k 10 400 python tools/train_bench.py --steps 6 --warmup 2 --ab DW_HIP > gpurun_out/r03_dw_ab.log 2>&1 || { tail -20 gpurun_out/r03_dw_ab.log; exit 1; }
tail -3 gpurun_out/r03_dw_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -k "fold" -q --timeout 300 --timeout-method thread > gpurun_out/r03_fold_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_fold_test.log
[ $rc -eq 0 ] || { grep -E "^E  |Error|FAILED" gpurun_out/r03_fold_test.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r03_bench_a.log 2>&1 || { tail -20 gpurun_out/r03_bench_a.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03_bench_a.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
for k, v in d["kernels"].items():
    print(f"  {k:14s} {v['median_us']:8.1f} us x{v['launches']}")
PY
