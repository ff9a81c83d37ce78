"""K-sweep of the bf16 GEMM at fixed M, N: separates the per-block fixed cost (prologue +
epilogue) from the per-K-tile main-loop cost.   python tools/gemm_sweep.py [N] [variant] [epi]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from recformer_amd._lib import set_knob  # noqa: E402
from tools.gemm_ab import timeit  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    set_knob("gemm_variant", int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    epi = int(sys.argv[3]) if len(sys.argv) > 3 else ops.RF_EPI_BIAS
    M = 65536
    dev = torch.device("cuda")
    for K in (64, 128, 256, 512, 768, 1536, 3072):
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16() * 0.05
        b = torch.randn(N, device=dev)
        t = timeit(lambda: ops.gemm(a, w, b, epi))
        tt = timeit(lambda: torch.matmul(a, w.t()))
        fl = 2 * M * N * K
        print(f"N={N} K={K:5d}: rf {t*1e6:7.1f}us {fl/t/1e12:6.0f}TF | hipBLASLt {tt*1e6:7.1f}us {fl/tt/1e12:6.0f}TF",
              flush=True)


if __name__ == "__main__":
    main()
