"""C2 forward steps (bench.py's workload: RecformerForSeqRec encode + score, 12L/768d, L = 1024, B = 64, fp32
parameters under autocast bf16) with library knobs from RF_KNOBS, for kernel traces of one setting per
process (tools/gpu/run.sh bandab):

    RF_KNOBS=band_path=3 python tools/c2_steps.py [steps] [warmup]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec, _lib  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):
        k, v = kv.split("=")
        _lib.set_knob(k, int(v))
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000))
    torch.manual_seed(0)
    m = RecformerForSeqRec(cfg).eval()
    m.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    m = m.to(dev)
    batch = {k: v.to(dev) for k, v in synth_batch(64, 1024, cfg.vocab_size, seed=100, item_len=21).items()}
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for _ in range(warm):
            m(**batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m(**batch)
        torch.cuda.synchronize()
    print(f"{os.environ.get('RF_KNOBS', '')}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
