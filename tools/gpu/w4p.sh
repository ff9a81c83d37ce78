#!/bin/bash
# the split-plane four-wave GEMM: parity, the C2 GEMM bar (w4p legs next to w4 and hipBLASLt), a same-process C2 A/B
set -o pipefail
O=gpurun_out/${1:-w4p}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py::test_gemm_split_plane_kernel > $O/pytest.log 2>&1 \
  || { grep -E "^E  |FAILED|Error" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/gemm_c2_bar.py gemm_w4p=1 > $O/bar.jsonl 2>&1 || { tail -20 $O/bar.jsonl; exit 1; }
grep shape $O/bar.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['leg'], d['us'], d['tflops'], d.get('bit_identical_to_default', ''))"
AB_AUTOCAST=1 timeout -k 10 400 python tools/ab_step.py knob:gemm_w4p 64 > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; exit 1; }
grep -E "ms/step|diff" $O/ab_c2.log
