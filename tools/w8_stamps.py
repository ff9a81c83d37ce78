"""Segment timeline of the eight-wave ping-pong GEMM (k_gemm_w8) from in-kernel s_memtime stamps: a
diagnostic build (tools/build_variant.sh w8st rf_gemm_w8.hip -DRF_W8_STAMPS, loaded with RF_HIP_LIB) makes
waves 0 (group 0) and 4 (group 1) stamp before and after every barrier. Per group and segment kind (load /
compute; epilogue-carrying load segments apart) it prints the mean cycles of work (previous barrier
release -> this barrier arrival) and of barrier wait (arrival -> release).

    RF_HIP_LIB=tools/varx/librf_w8st.so python tools/w8_stamps.py [N K epi]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from recformer_amd import _lib, ops  # noqa: E402

NS = 128


def run(N, K, epi):
    M = 65536
    dev = torch.device("cuda")
    lib = _lib.load()
    lib.rf_debug_gemm_stamps.argtypes = [ctypes.c_void_p]
    _lib.set_knob("gemm_w8", 1)
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
    b = torch.randn(N, device=dev, generator=g) * 0.02
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        ops.gemm(a, w, b, epi, out=out)
    buf = torch.zeros(256 * 2 * NS, dtype=torch.int64, device=dev)
    lib.rf_debug_gemm_stamps(ctypes.c_void_p(buf.data_ptr()))
    ops.gemm(a, w, b, epi, out=out)
    torch.cuda.synchronize()
    lib.rf_debug_gemm_stamps(ctypes.c_void_p(0))
    st = buf.view(256, 2, NS // 2, 2).cpu().numpy().astype(np.int64)  # [block][group][barrier][before/after]
    nk = K // 64
    print(f"M={M} N={N} K={K} epi={epi} (nk={nk})")
    for grp, first in ((0, 3), (1, 2)):  # barrier index of the first loop segment's end
        s = st[:, grp]
        nb = NS // 2
        work = s[:, 1:, 0] - s[:, :-1, 1]
        wait = s[:, 1:, 1] - s[:, 1:, 0]
        rows = {"load": [], "load+epi": [], "compute": []}
        m = 1 if grp == 0 else 0
        k = first
        while k + 1 < nb:
            kind = "load+epi" if (m % nk == 0 and m > 0) else "load"
            rows[kind].append(k - 1)
            rows["compute"].append(k)
            k += 2
            m += 1
        line = []
        for kind, idx in rows.items():
            idx = [i for i in idx if i < work.shape[1] and (s[:, i + 1, 1] > 0).all()]
            if not idx:
                continue
            line.append(f"{kind}: work {work[:, idx].mean():6.0f} wait {wait[:, idx].mean():6.0f} (n={len(idx)})")
        print(f"  group {grp}: " + " | ".join(line))
    span = st[:, :, -1, 1].max() - st[:, :, 0, 0].min()
    print(f"  stamped span (first {NS // 2} barriers) {span} cycles")


def main():
    args = [int(x) for x in sys.argv[1:4]] if len(sys.argv) > 3 else None
    cases = [tuple(args)] if args else [(2304, 768, ops.RF_EPI_BIAS), (3072, 768, ops.RF_EPI_BIAS_GELU),
                                        (3072, 768, ops.RF_EPI_NONE), (768, 3072, ops.RF_EPI_BIAS)]
    for N, K, epi in cases:
        run(N, K, epi)


if __name__ == "__main__":
    main()
