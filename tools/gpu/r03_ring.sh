#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "fold_mfma" -q --timeout 200 --timeout-method thread > gpurun_out/r03_ring.log 2>&1
rc=$?; tail -2 gpurun_out/r03_ring.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_ring.log | cut -c1-300 | head -20; exit 1; }
for q in 0 3; do
rm -rf gpurun_out/r03_gf/t; mkdir -p gpurun_out/r03_gf
RF_KNOBS=gfold_path=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_gf/t -o g -- python3 tools/gfold_bench.py > gpurun_out/r03_gf/log 2>&1 || { tail -20 gpurun_out/r03_gf/log; exit 1; }
echo "gfold_path $q"; grep "gfold c2\|gfold cat" gpurun_out/r03_gf/log
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
timeout -k 10 300 python tools/ab_knob.py gfold_path 0 3 > gpurun_out/r03_ring_ab.log 2>&1 || { tail -20 gpurun_out/r03_ring_ab.log; exit 1; }
tail -3 gpurun_out/r03_ring_ab.log | cut -c1-400
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -k "colsum or layernorm or c2_ or seqrec or lm_head" -q --timeout 200 --timeout-method thread > gpurun_out/r03_colsum.log 2>&1
rc=$?; tail -2 gpurun_out/r03_colsum.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_colsum.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > gpurun_out/r03_c3_g5.log 2>&1 || { tail -20 gpurun_out/r03_c3_g5.log; exit 1; }
tail -1 gpurun_out/r03_c3_g5.log
