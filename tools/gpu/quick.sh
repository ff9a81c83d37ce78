#!/bin/bash
# GPU check after a change: full -m gpu suite, then a short bench (per-step timing + kernels).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
for k, v in d["kernels"].items():
    print(f"  {k:12s} {v['avg_us']:8.1f} us x{v['launches']}")
PY
