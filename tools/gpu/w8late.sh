#!/bin/bash
# eight-wave GEMM: DMA waits in the compute segment (default build) vs all waits in the load segment (RF_W8_LATE)
set -o pipefail
O=gpurun_out/${1:-w8late}; mkdir -p $O
RF_HIP_LIB=tools/varx/librf_w8latest.so timeout -k 10 120 python tools/w8_stamps.py > $O/stamps_late.txt 2>&1 || { tail -20 $O/stamps_late.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_late.txt
for lib in recformer_amd/librecformer_hip.so tools/varx/librf_w8late.so; do
  RF_HIP_LIB=$lib timeout -k 10 300 python tools/gemm_c2_bar.py gemm_w8=1 > $O/bar_$(basename $lib .so).jsonl 2>&1 || { tail -20 $O/bar_$(basename $lib .so).jsonl; exit 1; }
  echo "== $lib"
  grep shape $O/bar_$(basename $lib .so).jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['leg'], d['us'], d['tflops'], d.get('bit_identical_to_default', ''))"
done
