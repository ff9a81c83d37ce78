"""Parity numbers per numerics mode at the C2 golden fixture (12L/768d, L=1024, B=2; the real
reference's fp32 outputs, tests/golden/c2_12l.npz): max / mean abs and rel-L2 of the 9 stored
hidden rows and the pooler, pooler cosine, score max-abs, top-10 agreement. One JSON line per mode.
    python tools/mode_errors.py"""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from recformer_amd import RecformerForSeqRec  # noqa: E402
from recformer_amd.hashinit import hash_tensor  # noqa: E402
from tests.common import BASE, batch_of, errs, hashed_model, load_golden  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = load_golden("c2_12l")
    for mode in ("fp32", "autocast_bf16", "autocast_fp16", "bf16_weights", "fp16_weights"):
        m = hashed_model(BASE, seed=2, cls=RecformerForSeqRec, item_num=1000)
        m.init_item_embedding(hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0))
        m = m.to(dev)
        if mode == "bf16_weights":
            m = m.to(torch.bfloat16)
        if mode == "fp16_weights":
            m = m.half()
        ctx = (torch.autocast("cuda", dtype=torch.bfloat16 if "bf16" in mode else torch.float16)
               if mode.startswith("autocast") else contextlib.nullcontext())
        batch = {k: v.to(dev) for k, v in batch_of(g).items()}
        with torch.no_grad(), ctx:
            out = m.longformer(**batch)
            scores = m(**batch)
        eh = errs(out.last_hidden_state[:, g["rows"]], g["hidden_rows"])
        ep = errs(out.pooler_output, g["pooler_output"])
        cos = F.cosine_similarity(out.pooler_output.float().cpu(), g["pooler_output"], dim=-1).min().item()
        top = scores.float().cpu().topk(10, dim=1).indices
        agree = min(len(set(top[b].tolist()) & set(g["scores"].topk(10, dim=1).indices[b].tolist()))
                    for b in range(top.shape[0]))
        print(json.dumps({"mode": mode, "hidden_rows": eh, "pooler": ep, "pooler_cos_min": cos,
                          "scores_max_abs": errs(scores, g["scores"])["max"], "top10_agree_min": agree}),
              flush=True)


if __name__ == "__main__":
    main()
