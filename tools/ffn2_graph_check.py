"""models.FFN2_LIBRARY under HIP-graph capture: GraphedForward with the flag on must replay the eager
scores with the flag on bit for bit, and stay within bf16 rounding of the rf_gemm path.

    python tools/ffn2_graph_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec, models  # noqa: E402
from recformer_amd.graphs import GraphedForward  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000))
    torch.manual_seed(0)
    m = RecformerForSeqRec(cfg).eval()
    m.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    m = m.to(dev)
    bb = {k: v.to(dev) for k, v in synth_batch(16, 1024, cfg.vocab_size, seed=216, item_len=21).items()}
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        models.FFN2_LIBRARY = False
        ref = m(**bb).float()
        models.FFN2_LIBRARY = True
        eager = m(**bb).float()
        g = GraphedForward(m, bb, check=False)
        rep = g(**bb).float()
        rep2 = g(**bb).float()
    torch.cuda.synchronize()
    print("graph replay == eager (flag on):", torch.equal(rep, eager), torch.equal(rep2, eager))
    d = (eager - ref).abs()
    print(f"flag on vs off: max-abs {d.max().item():.3e} mean {d.mean().item():.3e} "
          f"(score scale {ref.abs().mean().item():.3e}); top-1 agree "
          f"{(eager.argmax(-1) == ref.argmax(-1)).float().mean().item():.3f}")
    if not (torch.equal(rep, eager) and torch.equal(rep2, eager)):
        sys.exit(1)


if __name__ == "__main__":
    main()
