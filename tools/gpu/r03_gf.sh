#!/bin/bash
# per-kernel times of the fold path at the C2 shape (tools/gfold_bench.py under rocprofv3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03_gf
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k "fold" -q --timeout 100 --timeout-method thread > gpurun_out/r03_gf/test.log 2>&1 || { grep -E "^E  |FAILED" gpurun_out/r03_gf/test.log | head; exit 1; }
tail -1 gpurun_out/r03_gf/test.log
for q in 8 4 16; do
rm -rf gpurun_out/r03_gf/t
RF_KNOBS=gfold_qsplit=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_gf/t -o g -- python3 tools/gfold_bench.py > gpurun_out/r03_gf/log 2>&1 || { tail -20 gpurun_out/r03_gf/log; exit 1; }
echo "qsplit $q"; grep "gfold c2" gpurun_out/r03_gf/log
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r03_gf/t/**/*kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'gfold' in r['Kernel_Name']:
        d[(r['Kernel_Name'][:40], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k, v in sorted(d.items()):
    v.sort(); print(k, len(v), round(v[len(v)//2], 2))
PY
done
