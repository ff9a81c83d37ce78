#!/bin/bash
# A/B of GEMM library variants (tools/build_variant.sh), each in its own process, twice over.
# usage: tools/gpu/gemm_var.sh NAME...   (tools/var/librf_NAME.so; "prod" = the production build)
for rep in 1 2; do
  for n in "$@"; do
    if [ "$n" = prod ]; then lib=recformer_amd/librecformer_hip.so; else lib=tools/var/librf_$n.so; fi
    RF_HIP_LIB=$lib timeout -k 10 120 python3 tools/gemm_var.py || exit 1
  done
done
