"""Sweep a GEMM launch knob on the C2 layer shapes with their bench epilogues, interleaved repeats
in one process: the column-group width (gemm_gn: tiles of 256 columns per raster group) or the
kernel family (gemm_variant: 5 ping-pong, 6 four-wave).

    python tools/gemm_gn.py [values, default 2,3,4,6,12] [knob, default gemm_gn]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from recformer_amd._lib import set_knob  # noqa: E402
from tools.gemm_ab import timeit  # noqa: E402


def main():
    gns = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,3,4,6,12").split(",")]
    knob = sys.argv[2] if len(sys.argv) > 2 else "gemm_gn"
    default = {"gemm_gn": 6, "gemm_variant": 8, "gemm_pf": -1}[knob]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = 65536
    cases = [("qkv", 2304, 768, ops.RF_EPI_BIAS), ("out", 768, 768, ops.RF_EPI_BIAS),
             ("ffn1", 3072, 768, ops.RF_EPI_BIAS_GELU), ("ffn2", 768, 3072, ops.RF_EPI_BIAS)]
    for name, N, K, epi in cases:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * N * K
        res = {g: [] for g in gns}
        ref = None
        for rep in range(3):
            for g in gns:
                set_knob(knob, g)
                t = timeit(lambda: ops.gemm(a, w, b, epi, out=out), iters=30, warm=5)
                res[g].append(t)
                if ref is None:
                    ref = out.clone()
                else:
                    assert torch.equal(out, ref), (name, g)
        line = f"{name:5s} N={N} K={K}:"
        for g in gns:
            t = min(res[g])
            line += f"  {knob[5:]}={g} {t*1e6:6.1f}us {fl/t/1e12:5.0f}TF"
        tb = timeit(lambda: torch.matmul(a, w.t()), iters=30, warm=5)
        line += f"  | hipBLASLt (no epilogue) {tb*1e6:6.1f}us {fl/tb/1e12:5.0f}TF"
        print(line, flush=True)
    set_knob(knob, default)


if __name__ == "__main__":
    main()
