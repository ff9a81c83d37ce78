"""A/B of whole C2 steps in ONE process (clocks differ across devices and drift under load):
alternates blocks of steps between two settings of a models.py switch.

    python tools/ab_step.py [SWITCH] [B]      (default SWITCH=SPLIT_STREAM)

SWITCH = knob:NAME alternates the library knob NAME between 1 and 0 (recformer_amd._lib.set_knob),
e.g. knob:gemm_mfma32. AB_AUTOCAST=1: fp32 parameters under torch.autocast(bf16), bench.py's mode
(default: bf16 weights).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec, _lib, models  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    switch = sys.argv[1] if len(sys.argv) > 1 else "SPLIT_STREAM"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000))
    torch.manual_seed(0)
    m = RecformerForSeqRec(cfg).eval()
    m.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    autocast = os.environ.get("AB_AUTOCAST") == "1"
    for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):  # base knobs, e.g. gemm_mfma32=1
        k, v = kv.split("=")
        _lib.set_knob(k, int(v))
    m = m.to(dev) if autocast else m.to(dev).to(torch.bfloat16)

    def setv(val):
        if switch.startswith("knob:"):  # knob:NAME (1 / 0) or knob:NAME=a,b (a / b)
            name, _, vals = switch[5:].partition("=")
            a, b = (int(x) for x in vals.split(",")) if vals else (1, 0)
            _lib.set_knob(name, a if val else b)
        else:
            setattr(models, switch, val)
    batch = {k: v.to(dev) for k, v in synth_batch(B, 1024, cfg.vocab_size, seed=100, item_len=21).items()}
    res = {False: [], True: []}
    outs = {}
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        for rep in range(6):
            for val in (True, False):
                setv(val)
                for _ in range(2):
                    outs[val] = m(**batch)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    m(**batch)
                torch.cuda.synchronize()
                res[val].append((time.perf_counter() - t0) / 10 * 1e3)
    for val in (True, False):
        v = sorted(res[val])
        print(f"{switch}={val}: ms/step median {v[len(v) // 2]:.3f} min {v[0]:.3f} all {[round(x, 2) for x in res[val]]}")
    d = (outs[True] - outs[False]).abs()
    print(f"scores max-abs diff between settings {d.max().item():.3e} mean {d.mean().item():.3e}")


if __name__ == "__main__":
    main()
