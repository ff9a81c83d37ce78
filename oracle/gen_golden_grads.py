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

The reference's own mixed-precision drift (round 6): the same model, batch and loss run again under
CPU torch.autocast in bfloat16 and in float16 (the reference drivers train under torch.cuda.amp
autocast, finetune.py:106-110; CPU autocast is the same op-level cast policy), storing per parameter
the autocast gradient at the same slice positions and its relative L2 error against the fp32
gradient over the WHOLE tensor, plus the autocast loss and dL/dz. tests/test_gpu_train.py holds the HIP
autocast backward to a multiple of this drift per parameter group instead of fixed bounds.

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


def run(seq, batch, labels, dtype=None):
    """Loss, dL/dz and the parameter gradients (float64) of one fwd + bwd, optionally under CPU autocast."""
    keep = {}

    def hook(_mod, _inp, out):
        out.pooler_output.retain_grad()
        keep["z"] = out.pooler_output

    seq.zero_grad(set_to_none=True)
    hdl = seq.longformer.register_forward_hook(hook)
    if dtype is None:
        loss = seq(**batch, labels=labels)
    else:
        with torch.autocast("cpu", dtype=dtype):
            loss = seq(**batch, labels=labels)
    loss.backward()
    hdl.remove()
    grads = {n: p.grad.detach().double().flatten().clone() for n, p in seq.longformer.named_parameters()
             if p.grad is not None}
    return loss.detach().float(), keep["z"].grad.detach().float().clone(), grads


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
    loss, dz, grads = run(seq, batch, labels)
    arrays = {"loss": loss.numpy(), "dz": dz.numpy(), "labels": labels.numpy()}
    names = []
    for name, gr in grads.items():
        pos = slice_positions(gr.numel())
        names.append(name)
        arrays[f"g:{name}:norm"] = np.asarray(float(gr.norm()))
        arrays[f"g:{name}:maxabs"] = np.asarray(float(gr.abs().max()))
        arrays[f"g:{name}:pos"] = pos
        arrays[f"g:{name}:val"] = gr[torch.from_numpy(pos)].numpy().astype(np.float32)
    arrays["names"] = np.asarray(names)
    for tag, dt in (("bf16", torch.bfloat16), ("fp16", torch.float16)):
        l_ac, dz_ac, g_ac = run(seq, batch, labels, dt)
        arrays[f"ac_{tag}:loss"] = l_ac.numpy()
        arrays[f"ac_{tag}:dz"] = dz_ac.numpy()
        worst = 0.0
        for name in names:
            g32, ga = grads[name], g_ac[name]
            pos = torch.from_numpy(arrays[f"g:{name}:pos"])
            arrays[f"ac_{tag}:g:{name}:val"] = ga[pos].numpy().astype(np.float32)
            rel = float((ga - g32).norm() / g32.norm().clamp_min(1e-300))
            arrays[f"ac_{tag}:g:{name}:rel"] = np.asarray(rel)
            worst = max(worst, rel) if float(g32.abs().max()) > 1e-6 * float(arrays["g:" + name + ":maxabs"]) else worst
        print(f"autocast {tag}: loss {float(l_ac):.6f} (fp32 {float(loss):.6f}); max per-parameter rel-L2 drift {worst:.3e}")
    path = os.path.join(ROOT, "tests", "golden", "c2_grads.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB; loss", float(loss), "params", len(names))


if __name__ == "__main__":
    main()
