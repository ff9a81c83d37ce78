#!/bin/bash
# N-rank rehearsal of bench.py's distributed control flow on a one-GPU box: torchrun with 2 ranks
# sharing cuda:0, gloo collectives (RF_BENCH_REHEARSAL=1). Checks the launch, barriers,
# max-over-ranks timing and the single rank-0 JSON line; the numbers are not a scaling result.
set -o pipefail
mkdir -p gpurun_out
RF_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 \
  > gpurun_out/dist_rehearsal.log 2>&1
rc=$?
tail -3 gpurun_out/dist_rehearsal.log
exit $rc
