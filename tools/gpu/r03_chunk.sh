#!/bin/bash
# fold chunk rows adaptive to the grid + FFN2 L2 prefetch: fold / GEMM / training GPU tests, the C2
# bench line, C3 captured and C4 (4 per rank) captured steps.
set -o pipefail
O=gpurun_out/r03_chunk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_model.py -q --timeout 200 --timeout-method thread -k "fold or gemm or global or c2_ or pretrain or finetune" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" $O/tests.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > $O/c3_graph.log 2>&1 || { tail -20 $O/c3_graph.log; exit 1; }
tail -1 $O/c3_graph.log
timeout -k 10 300 python tools/pretrain_bench.py --batch 4 --steps 6 --warmup 2 --graph > $O/c4_b4.log 2>&1 || { tail -20 $O/c4_b4.log; exit 1; }
tail -1 $O/c4_b4.log
