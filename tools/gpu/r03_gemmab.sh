#!/bin/bash
# GEMM A/B (production vs variants in tools/varx/, each in its own process, alternated), then the
# -m gpu suite and a short bench.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for n in prod ${VARIANTS:-old}; do
    if [ "$n" = prod ]; then lib=recformer_amd/librecformer_hip.so; else lib=tools/varx/librf_$n.so; fi
    RF_HIP_LIB=$lib timeout -k 10 120 python3 tools/gemm_var.py || exit 1
  done
done 2>&1 | tee gpurun_out/gemmab.log
[ -n "$AB_ONLY" ] && exit 0
bash tools/gpu/quick.sh
