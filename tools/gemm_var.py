"""Time the layer GEMM shapes with the library named by RF_HIP_LIB (one variant per process;
tools/gpu/gemm_var.sh alternates variants) and print a checksum of each output so variants can
be checked for bit-identical results."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recformer_amd import ops  # noqa: E402
from tools.gemm_ab import timeit  # noqa: E402


def main():
    from recformer_amd import _lib
    for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):  # e.g. RF_KNOBS=gemm_mfma32=1
        k, v = kv.split("=")
        _lib.set_knob(k, int(v))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    for name, (M, N, K, epi) in {"qkv": (65536, 2304, 768, ops.RF_EPI_BIAS), "ffn1": (65536, 3072, 768, ops.RF_EPI_BIAS_GELU),
                                 "ffn2": (65536, 768, 3072, ops.RF_EPI_BIAS), "out": (65536, 768, 768, ops.RF_EPI_BIAS)}.items():
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        b = torch.randn(N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: ops.gemm(a, w, b, epi, out=out), iters=20, warm=5)
        h = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:10]
        res.append(f"{name} {t * 1e6:6.1f}us {2 * M * N * K / t / 1e12:5.0f}TF {h}")
    print(os.path.basename(os.environ.get("RF_HIP_LIB", "prod")), os.environ.get("RF_KNOBS", ""), " | ".join(res),
          flush=True)


if __name__ == "__main__":
    main()
