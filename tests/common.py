"""Shared test helpers: golden fixtures, hashed models, error metrics."""
import json
import os

import numpy as np
import torch

from recformer_amd import RecformerConfig, RecformerForSeqRec, RecformerModel
from recformer_amd.hashinit import hash_init_, hash_tensor
from recformer_amd.synth import BASE, C1, synth_batch  # noqa: F401

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BATCH_KEYS = ("input_ids", "attention_mask", "global_attention_mask", "token_type_ids",
              "item_position_ids")


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def batch_of(g):
    return {k: g[k] for k in BATCH_KEYS}


def hashed_model(kw, seed, cls=RecformerModel, **extra):
    cfg = RecformerConfig(**dict(kw, **extra))
    m = cls(cfg).eval()
    hash_init_(m if cls is RecformerModel else m.longformer, seed=seed)
    return m


def checksums(model):
    return {k: float(v.double().sum()) for k, v in model.state_dict().items() if v.is_floating_point()}


def errs(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    d = (a - b)
    return dict(max=float(d.abs().max()), mean=float(d.abs().mean()),
                rel=float(d.norm() / max(b.norm(), 1e-30)))


def hashed_pretrain(kw=C1, seed_lf=1, seed_head=6):
    """RecformerForPretraining with the golden fixture's weights (oracle/gen_golden.py)."""
    from recformer_amd import RecformerForPretraining
    m = RecformerForPretraining(RecformerConfig(**kw)).eval()
    hash_init_(m.longformer, seed=seed_lf)
    hash_init_(m.lm_head, seed=seed_head)
    return m


def pretrain_inputs(g):
    keys = [k for k in g if k.endswith("_a") or k.endswith("_b")]
    return {k: g[k] for k in keys}
