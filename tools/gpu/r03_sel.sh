#!/bin/bash
# Round 3: run a selection of GPU tests (args: pytest node ids / -k expressions), verbose, one process.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest "$@" -v --timeout 600 --timeout-method thread > gpurun_out/r03_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03_sel.log | tail -40
[ $rc -eq 0 ] || { grep -E "^E  " gpurun_out/r03_sel.log | cut -c1-300 | head -30; }
exit $rc
