#!/bin/bash
# full GPU suite, default bench (autocast bf16), fp16 bench, per-mode parity numbers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r02e_pytest.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r02e_pytest.log | tail -30; exit 1; }
tail -1 gpurun_out/r02e_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r02e_bench.log 2>&1 || { tail -20 gpurun_out/r02e_bench.log; exit 1; }
tail -1 gpurun_out/r02e_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --dtype fp16 --cpu-baseline-seconds 0 > gpurun_out/r02e_bench16.log 2>&1 || { tail -20 gpurun_out/r02e_bench16.log; exit 1; }
tail -1 gpurun_out/r02e_bench16.log | cut -c1-200
timeout -k 10 300 python tools/mode_errors.py > gpurun_out/r02e_modes.log 2>&1 || { tail -20 gpurun_out/r02e_modes.log; exit 1; }
cat gpurun_out/r02e_modes.log
