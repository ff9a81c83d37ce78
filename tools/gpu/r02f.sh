#!/bin/bash
# round-2 session f: GPU tests + smoke + bench, fold-overlap A/B, C3 global-backward A/B
set -o pipefail
mkdir -p gpurun_out
bash tools_gpu_round.sh || exit 1
timeout -k 10 300 python tools/ab_step.py FOLD_OVERLAP > gpurun_out/ab_overlap.log 2>&1 || exit 1
cat gpurun_out/ab_overlap.log
timeout -k 10 200 python tools/train_bench.py --steps 10 > gpurun_out/tb_merged.log 2>&1 || exit 1
timeout -k 10 200 python tools/train_bench.py --steps 10 --global-bwd-six > gpurun_out/tb_six.log 2>&1 || exit 1
tail -1 gpurun_out/tb_merged.log gpurun_out/tb_six.log
TRAIN_OUT=trainprof_f bash tools/gpu/trainprof.sh
