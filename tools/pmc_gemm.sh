#!/bin/bash
# PMC passes over one GEMM shape (separate --pmc runs; never combined with trace domains).
# usage: tools/pmc_gemm.sh M N K   (counter sets in $SETS, ';'-separated)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_${RF_GEMM_VARIANT:-0}_$$
mkdir -p $OUT
SETS=${SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM;SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"}
i=0
IFS=';' read -ra ARR <<< "$SETS"
for ctrs in "${ARR[@]}"; do
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT -o p$i -- python3 tools/gemm_one.py "$@" > /dev/null 2>&1
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gemm" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:34s} mean/dispatch {sum(v)/len(v):18.1f}  (n={len(v)})")
PY
