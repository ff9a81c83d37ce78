"""Same-process A/B of the four-wave GEMM's 256 x 192 tile (knob gemm_n192) on the training batch's
N = 768 shapes: median us per launch of each setting over alternating blocks.

    python tools/gemm_n192_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from recformer_amd._lib import set_knob  # noqa: E402


def block(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    for (M, N, K, epi) in [(16384, 768, 3072, ops.RF_EPI_BIAS), (16384, 768, 768, ops.RF_EPI_BIAS),
                           (16384, 768, 2304, ops.RF_EPI_NONE), (16384, 768, 3072, ops.RF_EPI_NONE),
                           (4096, 768, 768, ops.RF_EPI_BIAS)]:
        a = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.02).to(dev, torch.bfloat16)
        b = torch.randn(N, generator=g).to(dev)
        fn = lambda: ops.gemm(a, w, b if epi == ops.RF_EPI_BIAS else None, epi)  # noqa: E731
        res = {0: [], 1: []}
        for k in (0, 1):
            set_knob("gemm_n192", k)
            block(fn, 5)
        for rep in range(8):
            for k in (0, 1):
                set_knob("gemm_n192", k)
                res[k].append(block(fn))
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        fl = 2 * M * N * K
        print(f"M={M} N={N} K={K} epi={epi}: 256x256 {med[0]:.1f} us ({fl / med[0] / 1e6:.0f} TF/s), "
              f"256x192 {med[1]:.1f} us ({fl / med[1] / 1e6:.0f} TF/s)", flush=True)
    set_knob("gemm_n192", 1)


if __name__ == "__main__":
    main()
