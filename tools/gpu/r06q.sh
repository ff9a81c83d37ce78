#!/bin/bash
# round 6: the optimizer update overlapped with the backward (graphs.OVERLAP_OPTIMIZER) — graph / training
# parity, then a captured C3 A/B in one process
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_train.py \
  > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python tools/train_bench.py --graph --steps 8 --warmup 2 --ab graphs.OVERLAP_OPTIMIZER > $O/ab_c3.log 2>&1 \
  || { tail -5 $O/ab_c3.log; exit 1; }
tail -2 $O/ab_c3.log
