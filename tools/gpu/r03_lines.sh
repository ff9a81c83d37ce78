#!/bin/bash
# C5 retrieval / catalog lines (+ retrieval kernel trace), C3 captured / eager and C4 captured lines,
# C3 captured-step kernel trace: the non-headline artifacts of tools/gpu/r03_artifacts.sh.
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
timeout -k 10 300 python tools/retrieval_bench.py > $O/retrieval.log 2>&1 || { tail -20 $O/retrieval.log; exit 1; }
tail -4 $O/retrieval.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/retrieval_trace -o r -- python3 tools/retrieval_bench.py > $O/retrieval_trace.log 2>&1 || { tail -20 $O/retrieval_trace.log; exit 1; }
timeout -k 10 600 python tools/catalog_bench.py > $O/catalog.log 2>&1 || { tail -20 $O/catalog.log; exit 1; }
tail -2 $O/catalog.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --graph > $O/c3_graph.log 2>&1 || { tail -20 $O/c3_graph.log; exit 1; }
tail -1 $O/c3_graph.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 > $O/c3_eager.log 2>&1 || { tail -20 $O/c3_eager.log; exit 1; }
tail -1 $O/c3_eager.log
for b in 4 32; do
timeout -k 10 300 python tools/pretrain_bench.py --batch $b --steps 6 --warmup 2 --graph > $O/c4_b${b}_graph.log 2>&1 || { tail -20 $O/c4_b${b}_graph.log; exit 1; }
tail -1 $O/c4_b${b}_graph.log
done
TRAIN_OUT=$TAG/c3_graph_trace TRAIN_ARGS=--graph bash tools/gpu/trainprof.sh > $O/c3_graph_trace.txt 2>&1 || { tail -20 $O/c3_graph_trace.txt; exit 1; }
head -12 $O/c3_graph_trace.txt
