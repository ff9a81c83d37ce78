"""Run one GEMM shape repeatedly (for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (65536, 2304, 768)))
dev = torch.device("cuda")
a = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
b = torch.randn(N, device=dev)
for _ in range(10):
    ops.gemm(a, w, b, ops.RF_EPI_BIAS)
torch.cuda.synchronize()
