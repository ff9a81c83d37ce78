"""Our ping-pong GEMM vs hipBLASLt on square sizes (the guide's template is quoted at 4096^3 /
8192^3 on random operands) and on the layer shapes.   python tools/gemm_square.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import ops  # noqa: E402
from tools.gemm_ab import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in ((4096, 4096, 4096), (8192, 8192, 8192), (65536, 768, 3072), (65536, 3072, 768),
                      (65536, 2304, 768), (16384, 4096, 4096)):
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * N * K
        for rep in range(2):
            t = timeit(lambda: ops.gemm(a, w, None, ops.RF_EPI_NONE, out=out), iters=20, warm=5)
            tb = timeit(lambda: torch.matmul(a, w.t()), iters=20, warm=5)
            print(f"[{rep}] {M}x{N}x{K}: rf {t * 1e6:8.1f} us {fl / t / 1e12:6.0f} TF | hipBLASLt {tb * 1e6:8.1f} us "
                  f"{fl / tb / 1e12:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
