#!/bin/bash
# round-2 check: new ranker tests, the knob path, bench with defaults, bench --gpus 2 self-spawn
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ranker or rank_catalog or fold_h_paths or gfold" > gpurun_out/r02a_pytest.log 2>&1 || { tail -30 gpurun_out/r02a_pytest.log; exit 1; }
tail -2 gpurun_out/r02a_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r02a_bench.log 2>&1 || { tail -20 gpurun_out/r02a_bench.log; exit 1; }
tail -1 gpurun_out/r02a_bench.log | cut -c1-600
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --batch 8 --cpu-baseline-seconds 0 > gpurun_out/r02a_bench2.log 2>&1 || { tail -20 gpurun_out/r02a_bench2.log; exit 1; }
tail -1 gpurun_out/r02a_bench2.log | cut -c1-400
