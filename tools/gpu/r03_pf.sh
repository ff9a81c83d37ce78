#!/bin/bash
# L2 prefetch in the four-wave GEMM (knob gemm_pf): per-shape sweep at the C2 layer shapes, then a
# same-process C2 step A/B.
set -o pipefail
mkdir -p gpurun_out/r03_pf
O=gpurun_out/r03_pf
timeout -k 10 400 python tools/gemm_gn.py 0,1,2,3,4,258,260 gemm_pf > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
cat $O/sweep.log
timeout -k 10 300 python tools/ab_knob.py gemm_pf 0 ${PF:-2} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -4 $O/ab.log | cut -c1-600
