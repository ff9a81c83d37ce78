#!/bin/bash
# One GPU session: tests -> smoke -> bench -> rocprof kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest.log
grep -E "passed|failed|FAILED" gpurun_out/pytest.log | tail -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0 --no-kernel-timing > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
