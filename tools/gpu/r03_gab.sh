#!/bin/bash
# captured-step A/Bs of train.py switches (one graph per value, replays alternated in one process)
set -o pipefail
O=gpurun_out/r03_gab
mkdir -p $O
for f in ${FLAGS:-LN_BIAS_GRAD GLOBAL_QG_INSIDE}; do
timeout -k 10 400 python tools/train_bench.py --steps 6 --warmup 2 --graph --ab $f > $O/$f.log 2>&1 || { tail -20 $O/$f.log; exit 1; }
tail -2 $O/$f.log
done
