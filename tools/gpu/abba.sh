#!/bin/bash
# Order-balanced whole-step A/B of two library builds (A B B A, twice): per-process clocks and
# the position in a sequence of runs bias single-order comparisons by a few %.
#   tools/gpu/abba.sh tools/var/librf_X.so [recformer_amd/librecformer_hip.so]
# (variants: tools/build_variant.sh NAME SOURCE.hip -DFLAG=V)
A=$1
B=${2:-recformer_amd/librecformer_hip.so}
for l in "$A" "$B" "$B" "$A" "$A" "$B" "$B" "$A"; do
  RF_HIP_LIB=$l timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-baseline-seconds 0 \
    --no-kernel-timing 2>/dev/null |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$l'.split('/')[-1], d['value'], d['ms_per_step'])" ||
    exit 1
done
