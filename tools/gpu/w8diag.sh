#!/bin/bash
# eight-wave GEMM diagnosis: segment stamps (diagnostic build), then the PMC passes of w4 and w8
set -o pipefail
O=gpurun_out/${1:-w8diag}; mkdir -p $O
RF_HIP_LIB=tools/varx/librf_w8st.so timeout -k 10 120 python tools/w8_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt | grep -v amdgpu.ids
bash tools/gpu/pmc_w8.sh ${1:-w8diag}_pmc
