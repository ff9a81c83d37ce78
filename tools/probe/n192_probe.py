"""Diagnostic: the four-wave GEMM on 256 x 192 tiles (knob gemm_n192) against the 256 x 256 tile, per
epilogue and dtype: mismatch count, max |diff|, first mismatching (row, col)."""
import sys

import torch

sys.path.insert(0, ".")
from recformer_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    for dt in (torch.bfloat16, torch.float16):
        for (M, N, K) in ((4096, 3072, 768), (16384, 768, 768)):
            g = torch.Generator(device="cpu").manual_seed(5)
            a = (torch.randn(M, K, generator=g) * 0.5).to(dev, dt)
            w = (torch.randn(N, K, generator=g) * 0.05).to(dev, dt)
            b = torch.randn(N, generator=g).to(dev)
            out = {}
            for knob in (0, 1):
                _lib.set_knob("gemm_n192", knob)
                out[knob] = (ops.gemm(a, w, None, ops.RF_EPI_NONE), ops.gemm(a, w, b, ops.RF_EPI_BIAS))
            torch.cuda.synchronize()
            for name, x, y in zip(("none", "bias"), out[0], out[1]):
                d = (x.float() - y.float()).abs()
                bad = (x != y).nonzero()
                first = bad[:4].tolist() if bad.numel() else []
                print(f"{dt} M={M} N={N} K={K} {name}: mismatches {bad.shape[0]} max {float(d.max()):.3e} "
                      f"first {first}", flush=True)
            _lib.set_knob("gemm_n192", 1)


if __name__ == "__main__":
    main()
