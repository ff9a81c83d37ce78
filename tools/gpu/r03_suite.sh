#!/bin/bash
# the whole -m gpu suite and smoke (round-end gates)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${SUITE_ARGS:-} > gpurun_out/r03_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/r03_gpu_all.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_gpu_all.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1 || { tail -5 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
