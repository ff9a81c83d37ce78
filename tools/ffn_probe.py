"""Where the FFN1 GEMM loses against FFN2 (equal flops): the same M x N x K with each epilogue,
the transposed shape, and hipBLASLt, interleaved in one process (clock drift).

    python tools/ffn_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from tools.gemm_ab import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    M = 65536
    g = torch.Generator(device=dev).manual_seed(0)
    cases = []
    for (N, K) in ((3072, 768), (768, 3072), (2304, 768), (768, 768)):
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
        b = torch.randn(N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for name, epi in (("none", ops.RF_EPI_NONE), ("bias", ops.RF_EPI_BIAS), ("gelu", ops.RF_EPI_BIAS_GELU)):
            if epi == ops.RF_EPI_BIAS_GELU and N != 3072:
                continue
            cases.append((f"N={N} K={K} {name}", lambda a=a, w=w, b=b, epi=epi, out=out:
                          ops.gemm(a, w, None if epi == ops.RF_EPI_NONE else b, epi, out=out), 2 * M * N * K))
        cases.append((f"N={N} K={K} hipBLASLt", lambda a=a, w=w: torch.matmul(a, w.t()), 2 * M * N * K))
    for rep in range(2):
        for name, fn, fl in cases:
            t = timeit(fn, iters=30, warm=5)
            print(f"[{rep}] {name:28s} {t * 1e6:8.1f} us {fl / t / 1e12:7.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
