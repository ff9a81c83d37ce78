#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_graphs.py tests/test_gpu_pretrain.py -k "global_fold_bwd or c2_ or seqrec or captured or c4_pretrain_grads or dropout" -q --timeout 300 --timeout-method thread > gpurun_out/r03_gbwd.log 2>&1
rc=$?; tail -2 gpurun_out/r03_gbwd.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_gbwd.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 400 python tools/train_bench.py --steps 8 --warmup 2 --ab GLOBAL_BWD_HIP > gpurun_out/r03_gbwd_ab.log 2>&1 || { tail -20 gpurun_out/r03_gbwd_ab.log; exit 1; }
tail -2 gpurun_out/r03_gbwd_ab.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > gpurun_out/r03_gbwd_graph.log 2>&1 || { tail -20 gpurun_out/r03_gbwd_graph.log; exit 1; }
tail -1 gpurun_out/r03_gbwd_graph.log
timeout -k 10 300 python tools/pretrain_bench.py --batch 4 --steps 6 --warmup 2 --graph > gpurun_out/r03_gbwd_c4.log 2>&1 || { tail -20 gpurun_out/r03_gbwd_c4.log; exit 1; }
tail -1 gpurun_out/r03_gbwd_c4.log
