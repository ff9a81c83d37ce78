"""Micro-benchmark of the global-token path (rf_global_attn_fold_h_fwd) at the C2 shape
(B=64, Lp=1024, one global row each) and the catalog shape (B=4096 items, Lp=64).

    python tools/gfold_bench.py            # per-shape time of the whole fold path
    RF_HIP_LIB=... python tools/gfold_bench.py   # a diagnostic build of the library
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from tools.kbench import timeit  # noqa: E402

if os.environ.get("RF_GFOLD_GEMV"):  # tools/gpu/gf.sh: force the GEMV fold kernels
    from recformer_amd._lib import set_knob
    set_knob("gfold_path", 1)
for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):  # e.g. RF_KNOBS=gfold_qsplit=4
    from recformer_amd._lib import set_knob
    k, v = kv.split("=")
    set_knob(k, int(v))


def main():
    dev = torch.device("cuda")
    H, D = 12, 768
    g = torch.Generator(device="cpu").manual_seed(0)
    w = [(torch.randn(D, D, generator=g) * 0.03).bfloat16().to(dev) for _ in range(3)]
    b = [(torch.randn(D, generator=g) * 0.1).to(dev) for _ in range(3)]
    for name, B, Lp in (("c2", 64, 1024), ("catalog", 4096, 64)):
        pad = int(os.environ.get("RF_GF_PADCOLS", "0"))  # row stride D + pad (HBM channel-spread probe)
        h = torch.randn(B * Lp, D + pad, generator=g).bfloat16().to(dev)[:, :D]
        flags = torch.ones(B, Lp, dtype=torch.uint8, device=dev)
        flags[:, 0] = 2
        gidx = torch.zeros(B, 1, dtype=torch.int32, device=dev)
        out = torch.zeros(B * Lp, D, dtype=torch.bfloat16, device=dev)
        t = timeit(lambda: ops.global_attention_fold_h(h, w[0], b[0], 0.125, w[1], b[1], w[2], b[2], flags, gidx,
                                                       B, Lp, H, out), iters=30)
        print(f"gfold {name:8s} B={B} Lp={Lp}: {t*1e6:8.1f} us  out_sum={float(out[::Lp].float().sum()):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
