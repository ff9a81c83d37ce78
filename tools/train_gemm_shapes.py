"""The C3 training step's GEMM shapes (B=16 x L=1024 = 16384 token rows, d=768, FFN 3072) on the HIP
kernels next to hipBLASLt (torch.matmul, the same 16-bit operands, no epilogue) — where each training
GEMM stands against the library and against the dense MFMA peak.

    python tools/train_gemm_shapes.py

Prints one JSON line per shape: us per call (HIP events over 20 calls after 5 warm-up calls, each
timing in its own loop), TFLOP/s and the fraction of 2.5 PF for both."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402


def timed(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, D, F = 16384, 768, 3072

    def r(*shape, s=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * s).to(dt)

    lines = []
    # forward: C = A W^T (+ epilogue); dA: dC W (W^T stored, as the packed transposed copies)
    for name, (m, n, k), epi in (("fwd qkv", (M, 3 * D, D), ops.RF_EPI_BIAS),
                                 ("fwd out-proj", (M, D, D), ops.RF_EPI_BIAS),
                                 ("fwd ffn1 gelu+aux", (M, F, D), ops.RF_EPI_BIAS_GELU_AUX),
                                 ("fwd ffn2", (M, D, F), ops.RF_EPI_BIAS),
                                 ("dA qkv", (M, D, 3 * D), ops.RF_EPI_NONE),
                                 ("dA out-proj", (M, D, D), ops.RF_EPI_NONE),
                                 ("dA ffn2 (dgelu)", (M, F, D), ops.RF_EPI_DGELU),
                                 ("dA ffn1", (M, D, F), ops.RF_EPI_NONE)):
        a, w, b = r(m, k, s=0.5), r(n, k, s=0.05), torch.randn(n, device=dev, generator=g)
        aux = r(m, n) if epi in (ops.RF_EPI_BIAS_GELU_AUX, ops.RF_EPI_DGELU) else None
        bias = b if epi not in (ops.RF_EPI_NONE, ops.RF_EPI_DGELU) else None
        t_hip = timed(lambda: ops.gemm(a, w, bias, epi, resid=aux))
        wt = w.t()
        t_lib = timed(lambda: torch.matmul(a, wt))
        lines.append((name, m, n, k, t_hip, t_lib))
    # weight gradients dW = dC^T A (fp32 out)
    for name, (m, n, k) in (("dW qkv", (M, 3 * D, D)), ("dW out-proj", (M, D, D)), ("dW ffn1", (M, F, D)),
                            ("dW ffn2", (M, D, F))):
        dc, a = r(m, n, s=0.1), r(m, k, s=0.5)
        t_hip = timed(lambda: ops.weight_grad(dc, a))
        dct = dc.t()
        t_lib = timed(lambda: torch.matmul(dct, a).float())
        lines.append((name, m, n, k, t_hip, t_lib))
    for name, m, n, k, th, tl in lines:
        fl = 2.0 * m * n * k
        print(json.dumps({"gemm": name, "M": m, "N": n, "K": k, "hip_us": round(th, 1),
                          "hip_tflops": round(fl / th / 1e6, 1), "hip_frac": round(fl / th / 2.5e9, 3),
                          "hipblaslt_us": round(tl, 1), "hipblaslt_tflops": round(fl / tl / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
