#!/bin/bash
# Round 3: the new / changed GPU tests first, then the whole -m gpu suite, then a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pretrain.py "tests/test_gpu_kernels.py::test_rank_catalog_matches_restated_ranker" \
  "tests/test_gpu_kernels.py::test_retrieval_topk_argument_checks" "tests/test_gpu_train.py::test_train_mode_under_no_grad_applies_dropout" \
  "tests/test_gpu_train.py::test_seqrec_training_with_attention_dropout" -v --timeout 600 --timeout-method thread > gpurun_out/r03_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03_new.log | tail -30
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r03_new.log | head -40; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_all.log 2>&1
rc=$?
tail -5 gpurun_out/r03_all.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r03_all.log | head -40; exit $rc; }
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r03_bench.log 2>&1 || { tail -20 gpurun_out/r03_bench.log; exit 1; }
tail -1 gpurun_out/r03_bench.log | cut -c1-400
