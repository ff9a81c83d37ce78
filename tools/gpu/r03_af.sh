#!/bin/bash
# attention / fold change check: kernel + model + training GPU tests, then a short bench (per-kernel).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/af_tests.log 2>&1
rc=$?; tail -2 gpurun_out/af_tests.log; [ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/af_tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 0 > gpurun_out/af_bench.log 2>&1 || { tail -20 gpurun_out/af_bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/af_bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
print(" ".join(f"{k}={v['avg_us']:.1f}" for k, v in d["kernels"].items()))
PY
