"""Same-process GEMM bar at the C2 inference shapes (M = 65,536 token rows): hipBLASLt's plain
product (torch.mm, bf16 out, no epilogue) next to the HIP kernels without and with the bench's
epilogue, and any knob variants named on the command line. Legs alternate round-robin (3 rounds,
median per leg) so the clock drift under sustained MFMA load hits every leg alike.

    python tools/gemm_c2_bar.py [knob=value ...]      (one JSON line per shape and leg)

Operands are model-like (LayerNorm-scaled activations ~N(0,1), weights ~N(0, 0.02)): the clock the
chip holds depends on the data (MI355X_MICROARCH.md, DVFS item 1), so random +-1 operands would
rank the legs at a lower clock than the bench runs them.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import _lib, ops  # noqa: E402

SHAPES = {  # name: (N, K, epilogue, scale_cols) — the Linears of one layer
    "qkv": (2304, 768, ops.RF_EPI_BIAS, 768),
    "out": (768, 768, ops.RF_EPI_BIAS, 0),
    "ffn1": (3072, 768, ops.RF_EPI_BIAS_GELU, 0),
    "ffn2": (768, 3072, ops.RF_EPI_BIAS, 0),
}


def time_us(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    variants = [a.split("=") for a in sys.argv[1:]]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    M = 65536
    for name, (N, K, epi, sc) in SHAPES.items():
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.randn(N, device=dev, generator=g) * 0.02
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = None

        def ours(e, knobs=()):
            def f():
                ops.gemm(a, w, b if e != ops.RF_EPI_NONE else None, e, scale_cols=sc if e != ops.RF_EPI_NONE else 0,
                         col_scale=0.125 if sc else 1.0, out=out)
            return f

        b16 = b.bfloat16()
        legs = [("hipblaslt_plain", lambda: torch.mm(a, w.t(), out=out), ()),
                ("hipblaslt_bias", lambda: torch.addmm(b16, a, w.t(), out=out), ()),
                ("hip_plain", ours(ops.RF_EPI_NONE), ()),
                ("hip_epilogue", ours(epi), ())]
        for kv in variants:
            legs.append((f"hip_epilogue[{'='.join(kv)}]", ours(epi), (kv,)))
            legs.append((f"hip_plain[{'='.join(kv)}]", ours(ops.RF_EPI_NONE), (kv,)))
        times = {n: [] for n, _, _ in legs}
        hashes = {}
        for _ in range(3):
            for n, fn, knobs in legs:
                saved = []
                for k, v in knobs:
                    saved.append((k, _lib.get_knob(k)))
                    _lib.set_knob(k, int(v))
                times[n].append(time_us(fn))
                if n.startswith("hip_epilogue") and n not in hashes:
                    fn()
                    torch.cuda.synchronize()
                    hashes[n] = hash(out.view(torch.int16).cpu().numpy().tobytes())
                    if ref is None:
                        ref = out.float().clone()
                    else:
                        hashes[n + "_maxdiff"] = (out.float() - ref).abs().max().item()
                for k, v in saved:
                    _lib.set_knob(k, v)
        flop = 2 * M * N * K
        for n, _, _ in legs:
            t = statistics.median(times[n])
            rec = {"shape": name, "M": M, "N": N, "K": K, "leg": n, "us": round(t, 1),
                   "tflops": round(flop / t / 1e6, 1), "frac_2p5": round(flop / t / 1e6 / 2500, 4),
                   "all_us": [round(x, 1) for x in times[n]]}
            if n.startswith("hip_epilogue["):
                rec["bit_identical_to_default"] = hashes.get(n) == hashes.get("hip_epilogue")
                rec["max_abs_diff"] = hashes.get(n + "_maxdiff")
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
