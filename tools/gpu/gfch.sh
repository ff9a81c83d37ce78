# fold chunk-size A/B (tools/build_variant.sh chNNN rf_global.hip -DRF_GF_CH=NNN) under rocprofv3
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in prod ch128 ch64; do
  if [ $v = prod ]; then lib=$GRAFT_REPO_ROOT/recformer_amd/librecformer_hip.so; else lib=$GRAFT_REPO_ROOT/tools/var/librf_$v.so; fi
  RF_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gfch/$v -o k -- python3 tools/gfold_bench.py > gpurun_out/gfch_$v.log 2>&1
  python3 - $v <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/gfch/{sys.argv[1]}/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gfold' in r['Name']:
        print(sys.argv[1], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
  grep gfold gpurun_out/gfch_$v.log
done
