#!/bin/bash
# round 6: FFN2 on hipBLASLt (models.FFN2_LIBRARY) — C2 step A/B in one process (bench's autocast mode),
# graph capture with the flag on, and the GEMM bar with the library's bias epilogue
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
AB_AUTOCAST=1 timeout -k 10 300 python tools/ab_step.py FFN2_LIBRARY 64 > $O/ab_c2.log 2>&1 || { tail -5 $O/ab_c2.log; exit 1; }
tail -3 $O/ab_c2.log
timeout -k 10 200 python tools/ffn2_graph_check.py > $O/graph.log 2>&1 || { tail -5 $O/graph.log; exit 1; }
tail -3 $O/graph.log
timeout -k 10 300 python tools/gemm_c2_bar.py > $O/bar.jsonl 2>&1 || { tail -5 $O/bar.jsonl; exit 1; }
grep -E '"leg": "(hipblaslt|hip_epilogue)' $O/bar.jsonl
