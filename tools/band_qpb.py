"""Band attention: query blocks per workgroup (knob band_qpb) sweep at C2, one process.
    python tools/band_qpb.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from recformer_amd._lib import set_knob  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, L, H = 64, 1024, 12
    D = H * 64
    qkv = torch.randn(B * L, 3 * D, device=dev).bfloat16()
    flags = torch.ones(B, L, dtype=torch.uint8, device=dev)
    flags[:, 0] = 2
    gidx = torch.zeros(B, 1, dtype=torch.int32, device=dev)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:3 * D]
    ref = None
    for rep in range(2):
        for qpb in (2, 4, 8, 16):
            set_knob("band_qpb", qpb)
            out = ops.band_attention(q, k, v, flags, gidx, B, L, H, 32)
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref)
            t = timeit(lambda: ops.band_attention(q, k, v, flags, gidx, B, L, H, 32), iters=30, warm=5)
            print(f"[{rep}] qpb={qpb:2d}: {t * 1e6:6.1f} us {8 * B * L * D / t / 1e9:5.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
