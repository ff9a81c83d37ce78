"""Timeline of the C2 global-fold partial pass from the RF_GF_STAMPS build (tools/build_variant.sh
gfstamps rf_global.hip -DRF_GF_STAMPS=1): wave 0 of every (row, chunk) block records s_memrealtime
(100 MHz) at 16 points and the kernel copies them into the workspace's dropout-sum slots.

    RF_HIP_LIB=tools/varx/librf_gfstamps.so python tools/gfold_stamps.py

Points: 0 entry, 1 u + flags loaded, 2 first image DMA issued, then per 64-row sub-chunk s (0..3):
3+3s half A landed, 4+3s softmax done (before P.H), 5+3s P.H done + refill issued; 15 partials stored.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402


def a256(x):
    return (x + 255) & ~255


def main():
    dev = torch.device("cuda")
    H, D, B, Lp = 12, 768, 64, 1024
    g = torch.Generator(device="cpu").manual_seed(0)
    w = [(torch.randn(D, D, generator=g) * 0.03).bfloat16().to(dev) for _ in range(3)]
    b = [(torch.randn(D, generator=g) * 0.1).to(dev) for _ in range(3)]
    h = torch.randn(B * Lp, D, generator=g).bfloat16().to(dev)
    flags = torch.ones(B, Lp, dtype=torch.uint8, device=dev)
    flags[:, 0] = 2
    gidx = torch.zeros(B, 1, dtype=torch.int32, device=dev)
    ws = ops.global_fold_workspace(h, B, Lp, H, 1)
    R, nch = B, 4
    off = a256(R * 2 * 16 * D * 2) + a256(R * H * (D + 4) * 4) + 2 * a256(R * nch * 16 * 4)
    for _ in range(20):
        ops.global_attention_fold_h_stage(1, ws, h, w[0], b[0], 0.125, w[1], b[1], w[2], b[2], flags, gidx, B, Lp, H)
    torch.cuda.synchronize()
    runs = []
    for _ in range(5):
        ops.global_attention_fold_h_stage(1, ws, h, w[0], b[0], 0.125, w[1], b[1], w[2], b[2], flags, gidx, B, Lp, H)
        torch.cuda.synchronize()
        st = ws[off:off + R * nch * 16 * 4].view(torch.int32).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        runs.append(st.reshape(R * nch, 16))
    names = ["entry", "u loaded", "DMA issued"] + [f"s{s}:{p}" for s in range(4) for p in ("A landed", "softmax", "P.H")] + ["stored"]
    for k, t in enumerate(runs):
        t0 = t[:, 0].min()
        rel = (t - t0) * 0.01  # us
        print(f"run {k}: span {rel[:, 15].max():.2f} us; entry skew median {np.median(rel[:, 0]):.2f} max {rel[:, 0].max():.2f}")
        d = np.diff(rel, axis=1)
        for i in range(15):
            print(f"   {names[i]:>14s} -> {names[i + 1]:<14s} median {np.median(d[:, i]):6.2f}  p90 {np.percentile(d[:, i], 90):6.2f} us")


if __name__ == "__main__":
    main()
