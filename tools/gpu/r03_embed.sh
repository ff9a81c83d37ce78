#!/bin/bash
# Round 3: embedding-backward tests, the whole -m gpu suite, smoke, C3 step A/B of the HIP embedding
# backward and the C3 kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_optim.py -k "embedding_grad or embed_ln_bwd or adamw" -v --timeout 120 --timeout-method thread > gpurun_out/r03_emb.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_emb.log | tail -16
[ $rc -eq 0 ] || { grep -E "^E  " gpurun_out/r03_emb.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --ab EMBED_BWD_HIP > gpurun_out/r03_c3ab.log 2>&1 || { tail -20 gpurun_out/r03_c3ab.log; exit 1; }
tail -3 gpurun_out/r03_c3ab.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 > gpurun_out/r03_c3_hipadam.log 2>&1 || { tail -20 gpurun_out/r03_c3_hipadam.log; exit 1; }
tail -1 gpurun_out/r03_c3_hipadam.log
timeout -k 10 300 python tools/train_bench.py --steps 8 --warmup 2 --torch-adamw > gpurun_out/r03_c3_torchadam.log 2>&1 || { tail -20 gpurun_out/r03_c3_torchadam.log; exit 1; }
tail -1 gpurun_out/r03_c3_torchadam.log
TRAIN_OUT=r03_trainprof2 bash tools/gpu/trainprof.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/r03_gpu_all.log
[ $rc -eq 0 ] || { grep -E "^E  |FAILED" gpurun_out/r03_gpu_all.log | cut -c1-300 | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
