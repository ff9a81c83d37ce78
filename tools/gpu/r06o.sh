#!/bin/bash
# round 6: where k_rank_w32's candidate mode spends its time — variant libraries (flush / compaction
# compiled out; results wrong, timing only) traced on the 125k shard with the w32 family pinned
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base nofl noco; do
  lib=""; [ $v != base ] && lib=$PWD/tools/varx/librf_$v.so
  RF_HIP_LIB=$lib RF_KNOBS=rank_w32=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$v -o r -- \
    python3 tools/retrieval_bench.py --items 125000 > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  grep '"ms"' $O/t_$v.log | head -1 | cut -c1-150
done
