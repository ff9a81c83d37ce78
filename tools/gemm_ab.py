"""A/B the bf16 GEMM variants (knob gemm_variant) on the layer's shapes: correctness vs an fp32
torch reference, then time per variant and hipBLASLt (torch.matmul, no epilogue).

    python tools/gemm_ab.py [variants, default 1,5]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from recformer_amd._lib import set_knob  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,5").split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # correctness on ragged shapes first (every variant)
    for (M, N, K) in [(1000, 200, 128), (4000, 2056, 192), (4096, 2304, 768), (8000, 768, 3072), (4100, 2304, 64)]:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        b = torch.randn(N, device=dev)
        ref = a.float() @ w.float().t() + b
        for v in variants:
            set_knob("gemm_variant", v)
            out = ops.gemm(a, w, b, ops.RF_EPI_BIAS, out_f32=True)
            err = (out - ref).abs().max().item()
            print(f"check v{v} M={M} N={N} K={K}: max err {err:.3e}", flush=True)
            assert err < 1e-2 * K ** 0.5, err
    M = 65536
    cases = [("qkv3", 2304, 768, ops.RF_EPI_BIAS, False), ("out", 768, 768, ops.RF_EPI_BIAS_RESID, True),
             ("ffn1", 3072, 768, ops.RF_EPI_BIAS_GELU, False), ("ffn2", 768, 3072, ops.RF_EPI_BIAS_RESID, True)]
    for name, N, K, epi, f32 in cases:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16() * 0.05
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev) if epi == ops.RF_EPI_BIAS_RESID else None
        fl = 2 * M * N * K
        line = f"{name:5s} N={N} K={K}:"
        for v in variants:
            set_knob("gemm_variant", v)
            t = timeit(lambda: ops.gemm(a, w, b, epi, resid=r, out_f32=f32))
            line += f"  v{v} {t*1e6:7.1f}us {fl/t/1e12:6.0f}TF"
        tt = timeit(lambda: torch.matmul(a, w.t()))
        line += f"  | hipBLASLt {tt*1e6:7.1f}us {fl/tt/1e12:6.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
