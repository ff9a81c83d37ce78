#!/bin/bash
# round 6: w8 parity + bar + C2 A/B; the drift-anchored autocast training parity; the bench line with its batch sweep
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py::test_gemm_eight_wave_kernel tests/test_gpu_kernels.py::test_global_fold_fwd_stages_match_fused \
  tests/test_gpu_retrieval.py::test_shard_rank_large_k_few_overflows tests/test_gpu_train.py::test_side_stream_switches_bit_identical \
  > $O/pytest.log 2>&1 || { grep -E "^E  |FAILED|Error" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_train.py::test_c2_finetune_grads_match_reference" tests/test_gpu_train.py::test_c2_finetune_fp16_gradscaler_step \
  > $O/pytest_drift.log 2>&1; echo "drift tests rc=$?"; grep -E "passed|failed" $O/pytest_drift.log | tail -2
mkdir -p $O/drift && cp gpurun_out/drift/*.json $O/drift/ 2>/dev/null
timeout -k 10 300 python tools/gemm_c2_bar.py gemm_w8=1 > $O/bar.jsonl 2>&1 || { tail -20 $O/bar.jsonl; exit 1; }
grep shape $O/bar.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['leg'], d['us'], d['tflops'], d.get('bit_identical_to_default', ''))"
AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py knob:gemm_w8 64 > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; exit 1; }
grep -E "ms/step|diff" $O/ab_c2.log
timeout -k 10 400 python bench.py --cpu-baseline-seconds 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('batch_sweep')))"
