#!/bin/bash
# round 6: k_rank_w32 candidate mode without spills (LDS-staged candidates) — parity, then the C5 family A/B
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_retrieval.py \
  > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/retrieval_bench.py --family w16,w32 > $O/retrieval.log 2>&1 || { tail -5 $O/retrieval.log; exit 1; }
grep -E '"ms"' $O/retrieval.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RF_KNOBS=rank_w32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/retrieval_trace -o r -- \
  python3 tools/retrieval_bench.py --items 125000 > $O/retrieval_trace.log 2>&1 || { tail -5 $O/retrieval_trace.log; exit 1; }
