#!/bin/bash
# Ping-pong GEMM ablations (tools/micro/librf_diag{1,2,3,4,7}.so built with -DRF_GEMM_DIAG=n:
# 1 no LDS operand reads, 2 no operand DMA, 4 no barriers around the MFMA blocks), each in its
# own process at the FFN2 and FFN1 shapes, next to the production library.
for lib in recformer_amd/librecformer_hip.so tools/micro/librf_diag1.so tools/micro/librf_diag2.so tools/micro/librf_diag3.so tools/micro/librf_diag4.so tools/micro/librf_diag7.so; do
  RF_HIP_LIB=$lib timeout -k 10 60 python3 - "$lib" <<'PY'
import sys, torch
sys.path.insert(0, ".")
from recformer_amd import ops
from tools.gemm_ab import timeit
dev = torch.device("cuda")
res = []
for (M, N, K) in ((65536, 768, 3072), (65536, 3072, 768)):
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16(); w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    b = torch.randn(N, device=dev); out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.gemm(a, w, b, ops.RF_EPI_BIAS, out=out), iters=20, warm=5)
    res.append(f"{N}x{K}: {t*1e6:7.1f} us {2*M*N*K/t/1e12:6.0f} TF")
print(sys.argv[1].split("/")[-1], " | ".join(res), flush=True)
PY
done
