"""Generate tests/golden/c4_pretrain.npz: the REAL reference's pretraining step at C4 model size.

ORACLE / TEST INFRASTRUCTURE (build container only). Runs RecformerForPretraining from
/root/reference/recformer/models.py:370-520 (through oracle/ref_harness.py's three transformers-5.15
shims) at 12L/768d (longformer-base dims), B=2, view a at L=1024 (lengths 1024 / 700), view b at
L=128 (lengths 128 / 97), explicit masked-LM inputs and labels on both views, train mode with dropout
0, world size 1 — then backpropagates the total loss (contrastive CE + mlm_weight x the two masked-LM
CEs of LongformerLMHead over every token, models.py:492-510).

Masked-LM positions: the same number per sequence in each view (view a 96, view b 12), so that a
data-parallel split of the batch by sequence averages the per-rank masked-LM means to the full-batch
mean (tests/test_gpu_pretrain.py's world-2 check relies on it). Masked tokens are replaced by
<mask> = 50264 (the roberta/longformer vocabulary's mask id).

A second run of the same step under torch.autocast("cpu", dtype=torch.bfloat16) — the reference's
own mixed-precision run — stores its gradient slices and norms (prefix gb:) and loss, so the
16-bit parity tolerances are anchored on the drift of the reference's own bf16 run (e.g. its
value_global.bias gradients are only 0.97-0.99 cosine-close to its fp32 ones).

Stored: the loss, its contrastive part (the same call without MLM inputs), cl_correct_num, the
(2, 2) cosine logits, dL/dz1 and dL/dz2 (the pooled CLS vectors of the two views), and per parameter
of the whole model (encoder + lm_head) the gradient's L2 norm, max-abs and 256 entries at fixed flat
positions. Weights: recformer_amd/hashinit.py seeds (encoder 2, head 7), regenerated bit-exactly on
the GPU box. transformers 5.15 keeps lm_head.bias and lm_head.decoder.bias as two parameters (4.28
ties them; only decoder.bias is read in forward): the bias is copied into decoder.bias, and its
gradient is stored under decoder.bias (the build's tied lm_head.bias).

    python oracle/gen_golden_pretrain.py
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

from oracle.gen_golden_grads import slice_positions  # noqa: E402
from oracle.ref_harness import load_reference_models, make_reference_config  # noqa: E402
from recformer_amd.hashinit import hash_init_  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402

MASK_ID = 50264
N_MASK = {"a": 96, "b": 12}


def mlm_view(view, n, seed):
    """n masked positions per sequence among its valid tokens after <s>; labels -100 elsewhere."""
    g = torch.Generator().manual_seed(seed)
    ids = view["input_ids"].clone()
    labels = torch.full_like(ids, -100)
    for b in range(ids.shape[0]):
        valid = int(view["attention_mask"][b].sum())
        pos = 1 + torch.randperm(valid - 1, generator=g)[:n]
        labels[b, pos] = ids[b, pos]
        ids[b, pos] = MASK_ID
    return ids, labels


def inputs():
    va = synth_batch(2, 1024, BASE["vocab_size"], seed=52, lens=[1024, 700], item_len=21)
    vb = synth_batch(2, 128, BASE["vocab_size"], seed=53, lens=[128, 97], item_len=21)
    mia, mla = mlm_view(va, N_MASK["a"], 54)
    mib, mlb = mlm_view(vb, N_MASK["b"], 55)
    kw = {k + "_a": v for k, v in va.items()}
    kw.update({k + "_b": v for k, v in vb.items()})
    kw.update(mlm_input_ids_a=mia, mlm_labels_a=mla, mlm_input_ids_b=mib, mlm_labels_b=mlb)
    return kw


def main():
    torch.set_num_threads(os.cpu_count())
    M = load_reference_models()
    kw = dict(BASE, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    pre = M.RecformerForPretraining(make_reference_config(**kw))
    hash_init_(pre.longformer, seed=2)
    hash_init_(pre.lm_head, seed=7)
    with torch.no_grad():
        pre.lm_head.decoder.bias.copy_(pre.lm_head.bias)
    pre.train()
    batch = inputs()
    zs = []

    def hook(_m, _i, out):
        out.pooler_output.retain_grad()
        zs.append(out.pooler_output)

    hdl = pre.longformer.register_forward_hook(hook)
    out = pre(**batch)
    out.loss.backward()
    hdl.remove()
    z1, z2 = zs[0], zs[1]  # the view-a and view-b passes (models.py:410-436)
    with torch.no_grad():
        cl = pre(**{k: v for k, v in batch.items() if not k.startswith("mlm_")})
    arrays = {"loss": out.loss.detach().numpy(), "loss_contrastive": cl.loss.detach().numpy(),
              "cl_correct_num": out.cl_correct_num.numpy(), "logits": out.logits.detach().numpy(),
              "dz1": z1.grad.numpy(), "dz2": z2.grad.numpy(),
              **{k: v.numpy() for k, v in batch.items()}}
    names = []
    for name, p in pre.named_parameters():
        if p.grad is None:
            continue  # lm_head.bias of 5.15 (unused in forward; decoder.bias carries the gradient)
        gr = p.grad.detach().double().flatten()
        pos = slice_positions(gr.numel())
        names.append(name)
        arrays[f"g:{name}:norm"] = np.asarray(float(gr.norm()))
        arrays[f"g:{name}:maxabs"] = np.asarray(float(gr.abs().max()))
        arrays[f"g:{name}:pos"] = pos
        arrays[f"g:{name}:val"] = gr[torch.from_numpy(pos)].numpy().astype(np.float32)
    arrays["names"] = np.asarray(names)
    # the reference's own bf16-autocast step (drift anchor for the 16-bit tolerances)
    pre.zero_grad(set_to_none=True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out16 = pre(**batch)
    out16.loss.backward()
    arrays["loss_bf16"] = out16.loss.detach().float().numpy()
    for name, p in pre.named_parameters():
        if name in names:
            gr = p.grad.detach().double().flatten()
            arrays[f"gb:{name}:norm"] = np.asarray(float(gr.norm()))
            arrays[f"gb:{name}:val"] = gr[torch.from_numpy(arrays[f"g:{name}:pos"])].numpy().astype(np.float32)
    path = os.path.join(ROOT, "tests", "golden", "c4_pretrain.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB; loss", float(out.loss), "contrastive",
          float(cl.loss), "correct", int(out.cl_correct_num), "params", len(names))


if __name__ == "__main__":
    main()
