#!/bin/bash
# round 6: retrieval parity after the top-k change, then the C3 / C4 / C5 lines (tools/gpu/run.sh lines)
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_retrieval.py \
  > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/run.sh lines r06i_lines
