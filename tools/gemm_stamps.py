"""Timeline of the persistent ping-pong GEMM from in-kernel s_memtime stamps (diagnostic build
path: rf_debug_gemm_stamps). Per tile, wave 0 stamps: 0 start (K-tile 0 landed), 1 first P4
wait done, 2 first P8 wait done, 3 main loop end, 4 next prologue DMAs issued, 5 epilogue end.
    python tools/gemm_stamps.py [N K epi]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from recformer_amd import _lib, ops  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    epi = int(sys.argv[3]) if len(sys.argv) > 3 else ops.RF_EPI_BIAS
    M = 65536
    dev = torch.device("cuda")
    lib = _lib.load()
    lib.rf_debug_gemm_stamps.argtypes = [ctypes.c_void_p]
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16() * 0.05
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev) if epi in (ops.RF_EPI_BIAS_RESID,) else None
    f32 = r is not None
    for _ in range(3):
        ops.gemm(a, w, b, epi, resid=r, out_f32=f32)
    buf = torch.zeros(256 * 128, dtype=torch.int64, device=dev)
    lib.rf_debug_gemm_stamps(ctypes.c_void_p(buf.data_ptr()))
    ops.gemm(a, w, b, epi, resid=r, out_f32=f32)
    torch.cuda.synchronize()
    lib.rf_debug_gemm_stamps(ctypes.c_void_p(0))
    st = buf.view(256, 16, 8).cpu().numpy().astype(np.int64)
    ntile = (M // 256) * ((N + 255) // 256) // 256
    st = st[:, :ntile, :6]
    t0 = st[:, 0, 0].min()
    print(f"M={M} N={N} K={K} epi={epi}: {ntile} tiles per block")
    d = np.diff(st, axis=2)  # per tile segment durations
    names = ["start->P4w(1st)", "P4w->P8w(1st)", "P8w->loop end", "loop end->DMA issued", "epilogue"]
    for i, nm in enumerate(names):
        print(f"  {nm:22s} mean {d[:, :, i].mean():8.0f}  per-tile means {np.round(d[:, :, i].mean(0)).astype(int).tolist()}")
    gap = st[:, 1:, 0] - st[:, :-1, 5]
    print(f"  epilogue end -> next start mean {gap.mean():8.0f}  per-tile {np.round(gap.mean(0)).astype(int).tolist()}")
    tot = st[:, -1, 5] - st[:, 0, 0]
    print(f"  block span mean {tot.mean():.0f} min {tot.min()} max {tot.max()}; start skew {st[:, 0, 0].max() - t0}; "
          f"end skew {st[:, -1, 5].max() - st[:, -1, 5].min()}")


if __name__ == "__main__":
    main()
