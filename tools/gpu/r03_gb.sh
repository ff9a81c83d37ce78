#!/bin/bash
# global branch backward on rf_global_fold_bwd_full + rf_global_kv_grad: their tests, the training
# tests against the reference gradients, C3 captured and the C3 trace.
set -o pipefail
O=gpurun_out/r03_gb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_graphs.py tests/test_gpu_pretrain.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" $O/tests.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > $O/c3_graph.log 2>&1 || { tail -20 $O/c3_graph.log; exit 1; }
tail -1 $O/c3_graph.log
timeout -k 10 300 python tools/pretrain_bench.py --batch 4 --steps 6 --warmup 2 --graph > $O/c4_b4.log 2>&1 || { tail -20 $O/c4_b4.log; exit 1; }
tail -1 $O/c4_b4.log
TOPN=30 TRAIN_OUT=r03_gb/c3_trace TRAIN_ARGS=--graph bash tools/gpu/trainprof.sh > $O/c3_trace.txt 2>&1 || { tail -20 $O/c3_trace.txt; exit 1; }
head -32 $O/c3_trace.txt
