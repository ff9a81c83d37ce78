#!/bin/bash
# Fold partial kernel timing diagnostics (RF_GF_DIAG builds, tools/build_variant.sh): 1 no score
# MFMAs, 2 no refill DMA, 4 no P.H products, 5 = 1 + 4; per-kernel medians at the C2 shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_gfd
mkdir -p $O
for v in base gfd1 gfd2 gfd4 gfd5; do
rm -rf $O/t
if [ $v = base ]; then unset RF_HIP_LIB; else export RF_HIP_LIB=$GRAFT_REPO_ROOT/tools/var/librf_$v.so; fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o g -- python3 tools/gfold_bench.py > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
echo "== $v"; grep "gfold c2" $O/$v.log
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r03_gfd/t/**/*kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'gfold' in r['Kernel_Name']:
        d[(r['Kernel_Name'][:40], r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k, v in sorted(d.items()):
    v.sort(); print(k, len(v), round(v[len(v)//2], 2))
PY
done
