"""Small-batch serving latency: eager RecformerForSeqRec inference vs its HIP-graph replay
(graphs.GraphedForward), 12L/768d, bf16 weights, 10k-item scoring.

    python tools/graph_latency.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import GraphedForward, RecformerConfig, RecformerForSeqRec  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg)
    model.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    model = model.to(dev).to(torch.bfloat16).eval()
    for B, L in ((1, 1024), (4, 1024), (16, 1024), (1, 256)):
        b = {k: v.to(dev) for k, v in synth_batch(B, L, cfg.vocab_size, seed=1, item_len=21).items()}
        with torch.no_grad():
            te = timed(lambda: model(**b))
        g = GraphedForward(model, b)
        tg = timed(lambda: g(**b))
        tr = timed(lambda: g.graph.replay())
        print(json.dumps({"batch": B, "seq_len": L, "eager_ms": round(te * 1e3, 3), "graph_ms": round(tg * 1e3, 3),
                          "replay_only_ms": round(tr * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
