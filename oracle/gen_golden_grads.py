"""Generate tests/golden/c2_grads.npz: the REAL reference's finetune gradients at C2 dims.

ORACLE / TEST INFRASTRUCTURE (build container only). Runs RecformerForSeqRec from
/root/reference/recformer/models.py (through oracle/ref_harness.py's three transformers-5.15
shims) at 12L/768d, L=1024, B=2 — the c2_12l fixture's weights (hash seed 2), batch (seed 22,
lengths 1024 / 700), 1000-item catalog (seed 3) and labels [17, 923] — in train mode with dropout
0 (both probabilities), and backpropagates the full-softmax loss (models.py:586-591, the
finetune.sh setting). Stores the loss, dL/dz for the pooled CLS vectors, and per parameter the
gradient's L2 norm, max-abs and 256 entries at fixed flat positions (a checksum-like slice; the
full 148M gradients are not committed). Weights are regenerated bit-exactly on the GPU box from
the seeds (recformer_amd/hashinit.py).

    python oracle/gen_golden_grads.py
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
from recformer_amd.hashinit import hash_init_, hash_tensor  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402

NSLICE = 256


def slice_positions(numel: int) -> np.ndarray:
    """Fixed flat positions of a parameter's gradient slice: evenly spaced plus seeded draws."""
    g = np.random.default_rng(numel)
    even = np.linspace(0, numel - 1, NSLICE // 2).astype(np.int64)
    rnd = g.integers(0, numel, NSLICE - NSLICE // 2)
    return np.concatenate([even, rnd])


def main():
    torch.set_num_threads(os.cpu_count())
    M = load_reference_models()
    kw = dict(BASE, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    seq = M.RecformerForSeqRec(make_reference_config(item_num=1000, **kw))
    hash_init_(seq.longformer, seed=2)
    items = hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0)
    seq.init_item_embedding(items)
    seq.config.finetune_negative_sample_size = 0
    seq.train()
    batch = synth_batch(2, 1024, BASE["vocab_size"], seed=22, lens=[1024, 700], item_len=21)
    labels = torch.tensor([17, 923])
    keep = {}

    def hook(_mod, _inp, out):
        out.pooler_output.retain_grad()
        keep["z"] = out.pooler_output

    hdl = seq.longformer.register_forward_hook(hook)
    loss = seq(**batch, labels=labels)
    loss.backward()
    hdl.remove()
    arrays = {"loss": loss.detach().numpy(), "dz": keep["z"].grad.numpy(), "labels": labels.numpy()}
    names = []
    for name, p in seq.longformer.named_parameters():
        if p.grad is None:
            continue
        gr = p.grad.detach().double().flatten()
        pos = slice_positions(gr.numel())
        names.append(name)
        arrays[f"g:{name}:norm"] = np.asarray(float(gr.norm()))
        arrays[f"g:{name}:maxabs"] = np.asarray(float(gr.abs().max()))
        arrays[f"g:{name}:pos"] = pos
        arrays[f"g:{name}:val"] = gr[torch.from_numpy(pos)].numpy().astype(np.float32)
    arrays["names"] = np.asarray(names)
    path = os.path.join(ROOT, "tests", "golden", "c2_grads.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB; loss", float(loss), "params", len(names))


if __name__ == "__main__":
    main()
