#!/bin/bash
# round-2 session h: same-process C3 A/Bs of the global-backward switches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/train_bench.py --steps 5 --ab GLOBAL_BWD_DH16 > gpurun_out/ab_dh16.log 2>&1 || { tail -20 gpurun_out/ab_dh16.log; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 5 --ab GLOBAL_BWD_MERGED > gpurun_out/ab_merged.log 2>&1 || { tail -20 gpurun_out/ab_merged.log; exit 1; }
grep ms/step gpurun_out/ab_dh16.log gpurun_out/ab_merged.log
