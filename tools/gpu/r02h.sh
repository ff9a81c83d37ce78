#!/bin/bash
# round-2 session h: same-process C3 A/Bs of the global-backward switches (train_bench --ab)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/train_bench.py --steps 5 --ab GLOBAL_KV_BLOCKDIAG > gpurun_out/ab_kvbd.log 2>&1 || { tail -20 gpurun_out/ab_kvbd.log; exit 1; }
grep ms/step gpurun_out/ab_kvbd.log
