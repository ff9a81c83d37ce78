"""Run the C2 bench's four encoder GEMM shapes with their epilogues back to back (for rocprofv3 --pmc
passes and kernel traces of the GEMMs alone): qkv (65536 x 2304 x 768, bias + q-scale), out-proj
(65536 x 768 x 768, bias), FFN1 (65536 x 3072 x 768, bias + GELU), FFN2 (65536 x 768 x 3072, bias).
Operands at the bench's scales (activations ~N(0, 1) LayerNorm outputs, weights ~N(0, 0.02)), bf16.

    RF_KNOBS=name=v,... python tools/gemm_pmc.py [reps] [shape,...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402

SHAPES = {"qkv": (65536, 2304, 768, ops.RF_EPI_BIAS, 768), "out": (65536, 768, 768, ops.RF_EPI_BIAS, 0),
          "ffn1": (65536, 3072, 768, ops.RF_EPI_BIAS_GELU, 0), "ffn2": (65536, 768, 3072, ops.RF_EPI_BIAS, 0),
          # FFN1's shape with the plain bias epilogue: the GELU's share of FFN1 by difference
          "ffn1b": (65536, 3072, 768, ops.RF_EPI_BIAS, 0)}


def main():
    from recformer_amd import _lib
    for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):  # e.g. RF_KNOBS=gemm_w8=1
        k, v = kv.split("=")
        _lib.set_knob(k, int(v))
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    ops_ = []
    for n in names:
        M, N, K, epi, sc = SHAPES[n]
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.randn(N, device=dev, generator=g) * 0.02
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops_.append((n, a, w, b, epi, sc, out))
    for _ in range(reps):
        for n, a, w, b, epi, sc, out in ops_:
            ops.gemm(a, w, b, epi, scale_cols=sc, col_scale=0.125 if sc else 1.0, out=out, tag=f"gemm_{n}")
    torch.cuda.synchronize()
    print("ok", names, reps)


if __name__ == "__main__":
    main()
