#!/bin/bash
# rocprofv3 kernel-trace summary of the C3 training step (tools/train_bench.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${TRAIN_OUT:-trainprof}
rm -rf gpurun_out/$OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o tr -- python3 ${TRAIN_TOOL:-tools/train_bench.py} --steps 3 --warmup 1 ${TRAIN_ARGS:-} > gpurun_out/$OUT.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/' + __import__('os').environ.get('TRAIN_OUT', 'trainprof') + '/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("kernel ms per step", round(tot / 1e6 / 4, 2))
for r in rows[:int(__import__('os').environ.get('TOPN', '25'))]:
    print(f"{float(r['TotalDurationNs'])/tot*100:5.1f}% {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
PY
tail -1 gpurun_out/$OUT.log
