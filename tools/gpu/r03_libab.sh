#!/bin/bash
# Whole-step A/B of library builds: bench.py (C2) per build in its own process, alternated REPS times;
# prints seq/s and the per-kernel averages of the bench's timing pass. VARIANTS = names in tools/varx/.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for n in prod ${VARIANTS}; do
    if [ "$n" = prod ]; then lib=recformer_amd/librecformer_hip.so; else lib=tools/varx/librf_$n.so; fi
    RF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps ${STEPS:-100} --warmup 10 --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > gpurun_out/libab_$n.log 2>&1 || { tail -5 gpurun_out/libab_$n.log; exit 1; }
    python3 - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/libab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
ks = " ".join(f"{k}={v['avg_us']:.1f}" for k, v in d["kernels"].items())
print(f"{sys.argv[1]:10s} {d['value']:8.1f} seq/s {d['ms_per_step']:.3f} ms | {ks}", flush=True)
PY
  done
done 2>&1 | tee gpurun_out/libab.log
