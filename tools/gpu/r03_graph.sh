#!/bin/bash
# captured training step: tests, C3 eager vs graph
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_optim.py tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_graph_test.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r03_graph_test.log | tail -25
[ $rc -eq 0 ] || { grep -E "^E  " gpurun_out/r03_graph_test.log | cut -c1-300 | head -30; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 > gpurun_out/r03_c3_eager.log 2>&1 || { tail -20 gpurun_out/r03_c3_eager.log; exit 1; }
tail -1 gpurun_out/r03_c3_eager.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > gpurun_out/r03_c3_graph.log 2>&1 || { tail -20 gpurun_out/r03_c3_graph.log; exit 1; }
tail -1 gpurun_out/r03_c3_graph.log
