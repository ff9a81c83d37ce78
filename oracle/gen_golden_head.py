"""Generate tests/golden/c3_head.npz: the REAL reference's finetune scoring head at C3's catalog size.

ORACLE / TEST INFRASTRUCTURE (build container only). Runs RecformerForSeqRec.similarity_score and
its CrossEntropyLoss from /root/reference/recformer/models.py (through oracle/ref_harness.py) on a
10,000-item frozen catalog (init_item_embedding(vectors), models.py:533-537; hash seed 4) and 16
pooled vectors (hash seed 9): the full-softmax loss (models.py:586-588) and the sampled-softmax loss
on 1 + 127 fixed candidates per row (models.py:590-595 with the random negatives drawn here and
stored), each with dL/dz. The encoder is not run: the head is a function of the pooled vectors.

    python oracle/gen_golden_head.py
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.ref_harness import load_reference_models, make_reference_config  # noqa: E402
from recformer_amd.hashinit import hash_tensor  # noqa: E402
from recformer_amd.synth import C1  # noqa: E402

N_ITEMS, B, D, NEG = 10000, 16, 768, 127


def main():
    M = load_reference_models()
    kw = dict(C1, hidden_size=D, num_attention_heads=12, intermediate_size=4 * D)
    seq = M.RecformerForSeqRec(make_reference_config(item_num=N_ITEMS, **kw))
    items = hash_tensor("catalog", (N_ITEMS, D), "weight", seed=4, std=1.0)
    seq.init_item_embedding(items)
    z0 = hash_tensor("pooled", (B, D), "weight", seed=9, std=1.0)
    g = torch.Generator().manual_seed(5)
    labels = torch.randint(0, N_ITEMS, (B,), generator=g)
    labels[3] = labels[7]  # a shared label
    neg = torch.randint(0, N_ITEMS, (B, NEG), generator=g)
    cand = torch.cat([labels.unsqueeze(-1), neg], dim=-1)
    ce = torch.nn.CrossEntropyLoss()
    out = {"labels": labels.numpy(), "candidates": cand.numpy()}
    z = z0.clone().requires_grad_(True)
    logits = seq.similarity_score(z)
    loss = ce(logits, labels)
    loss.backward()
    out.update(loss_full=loss.detach().numpy(), dz_full=z.grad.numpy(), logits_rows=logits.detach()[:, :64].numpy())
    z = z0.clone().requires_grad_(True)
    logits = seq.similarity_score(z, cand)
    loss = ce(logits, torch.zeros_like(labels))
    loss.backward()
    out.update(loss_sampled=loss.detach().numpy(), dz_sampled=z.grad.numpy(), logits_sampled=logits.detach().numpy())
    path = os.path.join(ROOT, "tests", "golden", "c3_head.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
