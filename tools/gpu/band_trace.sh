#!/bin/bash
# band attention pipe2 (band_path 0) vs pipe3 (band_path 3): kernel traces of whole C2 steps, one setting per
# process, alternated twice (ABBA), per-kernel-tag averages side by side
set -o pipefail
O=gpurun_out/${1:-band_trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for run in 0a 3a 3b 0b; do
  bp=${run:0:1}
  RF_KNOBS=band_path=$bp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$run -o c2 -- \
    python3 tools/c2_steps.py 40 10 > $O/run_$run.log 2>&1 || { tail -5 $O/run_$run.log; exit 1; }
  grep ms/step $O/run_$run.log
  python3 tools/summarize_profile.py $O/trace_$run --config 64,1024,12 > $O/summary_$run.txt 2>&1 || true
done
python3 - <<PY
import json, re
rows = {}
for run in ("0a", "3a", "3b", "0b"):
    try:
        d = json.load(open("$O/trace_" + run + "/summary.json"))
    except Exception as ex:
        print(run, ex); continue
    for tag, v in d.get("tags", {}).items():
        rows.setdefault(tag, {})[run] = v.get("avg_us") or v.get("median_us")
print("tag".ljust(18), *[r.rjust(8) for r in ("0a", "3a", "3b", "0b")])
for tag, v in sorted(rows.items()):
    print(tag.ljust(18), *[("%8.1f" % v[r]) if v.get(r) else "       -" for r in ("0a", "3a", "3b", "0b")])
PY
