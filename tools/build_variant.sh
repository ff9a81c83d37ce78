#!/bin/bash
# Build a variant of librecformer_hip.so with extra compile flags for one source file (A/B on the
# GPU via RF_HIP_LIB, tools/gpu/gemm_var.sh):
#   tools/build_variant.sh NAME SOURCE.hip -DFLAG=V ...  ->  tools/var/librf_NAME.so
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../recformer_amd/csrc"
mkdir -p build/var ../../tools/var
objs=""
for f in rf_rowops rf_embed_bwd rf_gemm rf_gemm_w8 rf_gemm_tn rf_attn rf_attn_bwd rf_global rf_retrieval rf_optim rf_pack; do
  if [ "$f.hip" = "$src" ]; then
    # the retired GEMM main loops (knob gemm_variant 1-7) exist only in these A/B builds
    extra=""; [ "$f" = rf_gemm ] && extra="-DRF_GEMM_EXPERIMENTS"
    /opt/rocm/bin/hipcc $extra --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function "$@" -c $src -o build/var/${f}_$name.o
    objs="$objs build/var/${f}_$name.o"
  else
    objs="$objs build/$f.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/var/librf_$name.so $objs
