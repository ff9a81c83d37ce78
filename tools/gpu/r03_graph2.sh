#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_graph_test2.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_graph_test2.log | tail -8
[ $rc -eq 0 ] || { grep -E "^E  " gpurun_out/r03_graph_test2.log | cut -c1-300 | head -30; exit 1; }
for b in 4 32; do
timeout -k 10 300 python tools/pretrain_bench.py --batch $b --steps 6 --warmup 2 > gpurun_out/r03_c4_b${b}_eager.log 2>&1 || { tail -20 gpurun_out/r03_c4_b${b}_eager.log; exit 1; }
tail -1 gpurun_out/r03_c4_b${b}_eager.log
timeout -k 10 300 python tools/pretrain_bench.py --batch $b --steps 6 --warmup 2 --graph > gpurun_out/r03_c4_b${b}_graph.log 2>&1 || { tail -20 gpurun_out/r03_c4_b${b}_graph.log; exit 1; }
tail -1 gpurun_out/r03_c4_b${b}_graph.log
done
