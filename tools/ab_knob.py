"""A/B of a launch-path knob (recformer_amd._lib.set_knob) on whole C2 steps in ONE process — the
bench workload (12L/768d, B=64, L=1024, fp32 parameters under bf16 autocast, 10k-item scoring) —
alternating blocks of steps between the two values, plus the per-call-site kernel times (HIP events)
of each setting. Clocks differ across devices and drift under load, so only same-process
alternation is compared.

    python tools/ab_knob.py band_path 0 3 [B]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec, _lib, ops  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    knob, va, vb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000))
    torch.manual_seed(0)
    m = RecformerForSeqRec(cfg).eval()
    m.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    m = m.to(dev)
    batch = {k: v.to(dev) for k, v in synth_batch(B, 1024, cfg.vocab_size, seed=100, item_len=21).items()}
    res = {va: [], vb: []}
    kern = {va: {}, vb: {}}
    outs = {}
    old = _lib.set_knob(knob, va)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return m(**batch)

    with torch.no_grad():
        for _ in range(10):
            step()
        for rep in range(8):
            for val in (va, vb):
                _lib.set_knob(knob, val)
                for _ in range(2):
                    outs[val] = step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    step()
                torch.cuda.synchronize()
                res[val].append((time.perf_counter() - t0) / 10 * 1e3)
                ops.enable_timing(True)
                step()
                for k, v in ops.timing_results().items():
                    kern[val].setdefault(k, []).extend(v)
                ops.enable_timing(False)
    _lib.set_knob(knob, old)
    for val in (va, vb):
        v = sorted(res[val])
        ks = {k: round(1e3 * sorted(t)[len(t) // 2], 1) for k, t in sorted(kern[val].items())}
        print(f"{knob}={val}: ms/step median {v[len(v) // 2]:.3f} min {v[0]:.3f}; kernel medians us {ks}")
    d = (outs[va] - outs[vb]).abs()
    print(f"scores max-abs diff between settings {d.max().item():.3e}")


if __name__ == "__main__":
    main()
