#!/bin/bash
# Full -m gpu suite + smoke, C3 captured line and its kernel trace (top kernels per step).
set -o pipefail
mkdir -p gpurun_out/r03_check
O=gpurun_out/r03_check
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1
rc=$?; tail -2 $O/gpu_all.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" $O/gpu_all.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > $O/c3_graph.log 2>&1 || { tail -20 $O/c3_graph.log; exit 1; }
tail -1 $O/c3_graph.log
TOPN=40 TRAIN_OUT=r03_check/c3_trace TRAIN_ARGS=--graph bash tools/gpu/trainprof.sh > $O/c3_trace.txt 2>&1 || { tail -20 $O/c3_trace.txt; exit 1; }
head -45 $O/c3_trace.txt
timeout -k 10 300 python tools/ab_knob.py gemm_pf -1 0 > $O/ab_pf.log 2>&1 || { tail -20 $O/ab_pf.log; exit 1; }
tail -3 $O/ab_pf.log | cut -c1-500
timeout -k 10 400 python tools/train_bench.py --steps 8 --warmup 2 --ab-knob gemm_pf=-1,0 > $O/c3_ab_pf.log 2>&1 || { tail -20 $O/c3_ab_pf.log; exit 1; }
tail -3 $O/c3_ab_pf.log
