"""Per-kernel micro-benchmarks on the GPU (rf kernels vs torch/hipBLASLt where comparable).

    python tools/kbench.py [gemm|attn|all]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def gemm_bench():
    dev = torch.device("cuda")
    M = 65536
    cases = [("qkv3", 2304, 768, ops.RF_EPI_BIAS, False), ("qkv5", 3840, 768, ops.RF_EPI_BIAS, False),
             ("out", 768, 768, ops.RF_EPI_BIAS, False), ("ffn1", 3072, 768, ops.RF_EPI_BIAS_GELU, False),
             ("ffn2", 768, 3072, ops.RF_EPI_BIAS, False), ("ffn1_nogelu", 3072, 768, ops.RF_EPI_BIAS, False),
             ("ffn2_resid32", 768, 3072, ops.RF_EPI_BIAS_RESID, True)]
    for name, N, K, epi, f32 in cases:
        a = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev) if epi == ops.RF_EPI_BIAS_RESID else None
        t = timeit(lambda: ops.gemm(a, w, b, epi, resid=r, out_f32=f32))
        tt = timeit(lambda: torch.matmul(a, w.t()))
        fl = 2 * M * N * K
        print(f"gemm {name:12s} M={M} N={N} K={K}: rf {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF | "
              f"torch(hipBLASLt, no epilogue) {tt*1e6:8.1f} us {fl/tt/1e12:7.1f} TF", flush=True)


def attn_bench():
    dev = torch.device("cuda")
    B, L, H = 64, 1024, 12
    D = H * 64
    qkv = torch.randn(B * L, 5 * D, device=dev).bfloat16()
    flags = torch.ones(B, L, dtype=torch.uint8, device=dev)
    flags[:, 0] = 2
    gidx = torch.zeros(B, 1, dtype=torch.int32, device=dev)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:3 * D]
    t = timeit(lambda: ops.band_attention(q, k, v, flags, gidx, B, L, H, 32))
    nbytes = 8 * B * L * D
    print(f"band_attn B={B} L={L}: {t*1e6:.1f} us, {nbytes/t/1e9:.0f} GB/s algorithmic", flush=True)
    ctx = torch.empty(B * L, D, device=dev, dtype=torch.bfloat16)
    qg = torch.randn(B, D, device=dev).bfloat16()
    t = timeit(lambda: ops.global_attention(qg, qkv[:, 3 * D:4 * D], qkv[:, 4 * D:], flags, gidx, B, L, H, ctx))
    print(f"global_attn (reference structure, kg/vg precomputed) B={B} L={L}: {t*1e6:.1f} us", flush=True)
    h = qkv[:, :D]
    w = (torch.randn(2 * D, D, device=dev) * 0.05).bfloat16()
    bb = torch.zeros(2 * D, device=dev)
    t = timeit(lambda: ops.global_attention_fold(qg, h, w[:D], bb[:D], w[D:], bb[D:], flags, gidx, B, L, H, ctx))
    print(f"global_attn_fold B={B} L={L}: {t*1e6:.1f} us (reads h once: {B*L*D*2/t/1e9:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("gemm", "all"):
        gemm_bench()
    if what in ("attn", "all"):
        attn_bench()
