#!/bin/bash
# PMC passes of the four C2 GEMMs alone, the four-wave and the eight-wave kernels (tools/gpu/run.sh gemmpmc, twice)
set -o pipefail
for v in 0 1; do
  RF_KNOBS=gemm_w8=$v bash tools/gpu/run.sh gemmpmc ${1:-pmcw8}_w$v > /dev/null 2>&1 || { echo "gemmpmc w8=$v failed"; tail -5 gpurun_out/${1:-pmcw8}_w$v/*.log; exit 1; }
  echo "== gemm_w8=$v"; cat gpurun_out/${1:-pmcw8}_w$v/summary.txt
done
