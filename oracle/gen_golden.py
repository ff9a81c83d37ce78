"""Generate tests/golden/*.npz from the REAL reference (build container only).

ORACLE / TEST INFRASTRUCTURE. Runs recformer/models.py from /root/reference through
oracle/ref_harness.py (3 runtime shims, transformers 5.15) on synthetic inputs with
hash-generated weights (recformer_amd/hashinit.py), and stores inputs + outputs. The
fixtures are data (no reference source); weights are regenerated bit-exactly from the
seed by the tests, and per-parameter checksums are stored to prove it.

    python oracle/gen_golden.py            # writes tests/golden/
    python oracle/gen_golden.py attn       # only the output_attentions fixtures
"""
from __future__ import annotations

import json
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
from recformer_amd.synth import BASE, C1, synth_batch  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

def checksums(model):
    return {k: float(v.double().sum()) for k, v in model.state_dict().items() if v.is_floating_point()}


def run_model(M, kw, seed, batch, extra=None):
    ref = M.RecformerModel(make_reference_config(**kw)).eval()
    hash_init_(ref, seed=seed)
    with torch.no_grad():
        out = ref(**batch)
    return ref, out


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


def attention_fixtures(M):
    """c1_attn_{ragged,l200}.npz: output_attentions=True of the reference on the c1_ragged / c1_l200
    inputs (same batches, weight seed 1): per layer l, attentions `a{l}` (B,H,L,G+2w+1) and
    global_attentions `g{l}` (B,H,Lp,G)."""
    for name, v in (("ragged", dict(B=4, L=256, lens=[256, 200, 131, 77],
                                    extra=((0, 5), (1, 100), (1, 150), (2, 140)))),
                    ("l200", dict(B=4, L=200, lens=[200, 150, 64, 1], extra=()))):
        batch = synth_batch(v["B"], v["L"], C1["vocab_size"], seed=11, lens=v["lens"],
                            extra_globals=v["extra"])
        ref = M.RecformerModel(make_reference_config(**C1)).eval()
        hash_init_(ref, seed=1)
        with torch.no_grad():
            out = ref(**batch, output_attentions=True)
        arrays = {}
        for i, (a, g) in enumerate(zip(out.attentions, out.global_attentions)):
            arrays[f"a{i}"], arrays[f"g{i}"] = a, g
        save(f"c1_attn_{name}.npz", **arrays)


def main():
    torch.set_num_threads(os.cpu_count())
    M = load_reference_models()
    if sys.argv[1:] == ["attn"]:
        attention_fixtures(M)
        return
    manifest = {}

    # --- C1 variants -----------------------------------------------------------------
    variants = {
        "c1_full": dict(B=4, L=256, lens=None, extra=()),
        "c1_ragged": dict(B=4, L=256, lens=[256, 200, 131, 77], extra=((0, 5), (1, 100), (1, 150), (2, 140))),
        "c1_l200": dict(B=4, L=200, lens=[200, 150, 64, 1], extra=()),
    }
    for name, v in variants.items():
        batch = synth_batch(v["B"], v["L"], C1["vocab_size"], seed=11, lens=v["lens"],
                            extra_globals=v["extra"])
        ref, out = run_model(M, C1, 1, batch)
        save(f"{name}.npz", last_hidden_state=out.last_hidden_state, pooler_output=out.pooler_output,
             **batch)
        manifest[name] = dict(config="C1", weight_seed=1, checksums=checksums(ref))

    # --- 12L/768d, L=1024, B=2 + scoring + SeqRec losses ------------------------------
    batch = synth_batch(2, 1024, BASE["vocab_size"], seed=22, lens=[1024, 700], item_len=21)
    seq = M.RecformerForSeqRec(make_reference_config(item_num=1000, **BASE)).eval()
    hash_init_(seq.longformer, seed=2)
    items = hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0)
    seq.init_item_embedding(items)
    with torch.no_grad():
        out = seq.longformer(**batch)
        scores = seq(**batch)
        labels = torch.tensor([17, 923])
        seq.config.finetune_negative_sample_size = 0
        loss_full = seq(**batch, labels=labels)
        cand = torch.cat([labels.unsqueeze(-1), torch.randint(0, 1000, (2, 64), generator=torch.Generator().manual_seed(5))], -1)
        s_cand = seq.similarity_score(out.pooler_output, cand)
        loss_samp = torch.nn.functional.cross_entropy(s_cand, torch.zeros(2, dtype=torch.long))
    rows = torch.tensor([0, 1, 31, 32, 33, 511, 699, 700, 1023])
    save("c2_12l.npz", pooler_output=out.pooler_output, hidden_rows=out.last_hidden_state[:, rows],
         rows=rows, scores=scores, labels=labels, loss_full=loss_full, candidates=cand,
         scores_cand=s_cand, loss_sampled=loss_samp, **batch)
    manifest["c2_12l"] = dict(config="BASE", weight_seed=2, item_seed=3,
                              checksums=checksums(seq.longformer))

    # --- 1 layer at 768d: fp32 and the reference's own bf16 autocast ---------------------
    one = dict(BASE, num_hidden_layers=1, attention_window=[64])
    batch = synth_batch(2, 128, BASE["vocab_size"], seed=33, lens=[128, 90], item_len=21)
    ref, out = run_model(M, one, 4, batch)
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        out16 = ref(**batch)
    # the reference's own bf16-autocast drift vs its fp32 run calibrates the bf16 tolerance
    d = (out16.last_hidden_state.float() - out.last_hidden_state)
    ref_bf16_drift = torch.tensor([d.abs().max(), d.abs().mean(),
                                   d.norm() / out.last_hidden_state.norm()])
    save("l1_768.npz", last_hidden_state=out.last_hidden_state, ref_bf16_drift=ref_bf16_drift,
         **batch)
    manifest["l1_768"] = dict(config="BASE-1L", weight_seed=4, checksums=checksums(ref))

    # --- pretraining (A10): two views + MLM, world size 1 -----------------------------------
    pre = M.RecformerForPretraining(make_reference_config(**C1)).eval()
    hash_init_(pre.longformer, seed=1)
    hash_init_(pre.lm_head, seed=6)
    with torch.no_grad():  # 4.28 ties decoder.bias to lm_head.bias; 5.15 keeps two: make them equal
        pre.lm_head.decoder.bias.copy_(pre.lm_head.bias)
    va = synth_batch(4, 256, C1["vocab_size"], seed=44, lens=[256, 180, 97, 40])
    vb = synth_batch(4, 64, C1["vocab_size"], seed=45, lens=[64, 33, 64, 12])
    g = torch.Generator().manual_seed(46)

    def mlm(view, mask_id=3):
        ids = view["input_ids"].clone()
        sel = (torch.rand(ids.shape, generator=g) < 0.15) & (view["attention_mask"] == 1)
        sel[:, 0] = False
        labels = torch.where(sel, ids, torch.full_like(ids, -100))
        return torch.where(sel, torch.full_like(ids, mask_id), ids), labels

    mia, mla = mlm(va)
    mib, mlb = mlm(vb)
    sfx = lambda d, x: {k + "_" + x: v for k, v in d.items()}  # noqa: E731
    with torch.no_grad():
        out = pre(**sfx(va, "a"), **sfx(vb, "b"), mlm_input_ids_a=mia, mlm_labels_a=mla,
                  mlm_input_ids_b=mib, mlm_labels_b=mlb)
        out_nomlm = pre(**sfx(va, "a"), **sfx(vb, "b"))
    save("c1_pretrain.npz", loss=out.loss, logits=out.logits, cl_correct_num=out.cl_correct_num,
         loss_contrastive=out_nomlm.loss, mlm_input_ids_a=mia, mlm_labels_a=mla, mlm_input_ids_b=mib,
         mlm_labels_b=mlb, **sfx(va, "a"), **sfx(vb, "b"))
    manifest["c1_pretrain"] = dict(config="C1", weight_seed=1, head_seed=6,
                                   checksums=checksums(pre))

    # state-dict layout of the drop-in classes
    layout = {}
    for cls in ("RecformerModel", "RecformerForSeqRec", "RecformerForPretraining"):
        m = getattr(M, cls)(make_reference_config(**C1))
        layout[cls] = {k: [list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()}
    manifest["state_dict_layout_C1"] = layout

    attention_fixtures(M)

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote manifest")


if __name__ == "__main__":
    main()
