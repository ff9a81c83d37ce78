"""Tier (i): the CPU restatement (oracle/restatement.py) against golden fixtures made by
the real reference (oracle/gen_golden.py). Pins the oracle before it is trusted."""
import pytest
import torch

from oracle import restatement as R
from tests.common import (BASE, C1, batch_of, checksums, errs, hashed_model, load_golden,
                          manifest)
from recformer_amd.hashinit import hash_tensor


@pytest.mark.parametrize("name", ["c1_full", "c1_ragged", "c1_l200"])
def test_c1_variants(name):
    g = load_golden(name)
    m = hashed_model(C1, seed=1)
    assert checksums(m) == pytest.approx(manifest()[name]["checksums"], rel=0, abs=1e-9)
    h, p = R.model_forward(m.state_dict(), m.config, **batch_of(g))
    assert h.shape == g["last_hidden_state"].shape
    assert errs(h, g["last_hidden_state"])["max"] <= 1e-5
    assert errs(p, g["pooler_output"])["max"] <= 1e-5


def test_one_layer_768():
    g = load_golden("l1_768")
    m = hashed_model(dict(BASE, num_hidden_layers=1, attention_window=[64]), seed=4)
    assert checksums(m) == pytest.approx(manifest()["l1_768"]["checksums"], rel=0, abs=1e-6)
    h, _ = R.model_forward(m.state_dict(), m.config, **batch_of(g))
    assert errs(h, g["last_hidden_state"])["max"] <= 1e-5


@pytest.mark.slow
def test_12l_768_scores_and_losses():
    torch.set_num_threads(8)
    g = load_golden("c2_12l")
    m = hashed_model(BASE, seed=2)
    h, p = R.model_forward(m.state_dict(), m.config, **batch_of(g))
    assert errs(p, g["pooler_output"])["max"] <= 1e-4
    assert errs(h[:, g["rows"]], g["hidden_rows"])["max"] <= 1e-4
    items = hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0)
    s = R.cosine_scores(p, items, 0.05)
    assert errs(s, g["scores"])["max"] <= 1e-3
    assert abs(float(R.seqrec_loss(s, g["labels"])) - float(g["loss_full"])) <= 1e-4
    sc = R.cosine_scores(p, items[g["candidates"]], 0.05)
    assert errs(sc, g["scores_cand"])["max"] <= 1e-3
    assert abs(float(R.seqrec_loss(sc, torch.zeros(2, dtype=torch.long))) - float(g["loss_sampled"])) <= 1e-4


def test_pretrain_two_views_mlm():
    """A10: RecformerForPretraining loss / cos logits / correct count vs the reference run."""
    from tests.common import hashed_pretrain
    g = load_golden("c1_pretrain")
    m = hashed_pretrain()
    assert checksums(m) == pytest.approx(manifest()["c1_pretrain"]["checksums"], rel=0, abs=1e-9)
    cfg = m.config
    sd_lf = m.longformer.state_dict()
    sd_head = m.lm_head.state_dict()
    va = {k[:-2]: g[k] for k in ("input_ids_a", "attention_mask_a", "global_attention_mask_a",
                                 "token_type_ids_a", "item_position_ids_a")}
    vb = {k[:-2]: g[k] for k in ("input_ids_b", "attention_mask_b", "global_attention_mask_b",
                                 "token_type_ids_b", "item_position_ids_b")}
    loss, cos, correct = R.pretrain_forward(sd_lf, sd_head, cfg, va, vb, g["mlm_input_ids_a"], g["mlm_labels_a"],
                                            g["mlm_input_ids_b"], g["mlm_labels_b"])
    assert abs(float(loss) - float(g["loss"])) <= 1e-5
    assert errs(cos, g["logits"])["max"] <= 1e-4
    assert int(correct) == int(g["cl_correct_num"])
    loss0, _, _ = R.pretrain_forward(sd_lf, sd_head, cfg, va, vb)
    assert abs(float(loss0) - float(g["loss_contrastive"])) <= 1e-5


@pytest.mark.parametrize("case", ["ties", "masked", "cosine"])
def test_ranker_restatement_matches_reference(case):
    """utils.py:76-108 restated (oracle.restatement.ranker_metrics) vs the real Ranker's outputs
    (tests/golden/ranker.npz, oracle/gen_golden_ranker.py): ties, -MAX_VAL entries, B = 37."""
    g = load_golden("ranker")
    ks = [int(k) for k in g["ks"]]
    got = R.ranker_metrics(g[f"{case}_scores"].clone(), g[f"{case}_labels"].clone(), ks)
    ref = g[f"{case}_metrics"].tolist()
    assert len(got) == len(ref)
    for a, b in zip(got[:-1], ref[:-1]):
        assert a == pytest.approx(b, abs=1e-7)
    assert got[-1] == pytest.approx(ref[-1], rel=1e-6)


@pytest.mark.parametrize("case", ["ragged", "l200"])
def test_attention_probs_match_reference(case):
    """The restatement's attention probabilities (band_global_attention probs_out) against the
    reference's output_attentions=True run (oracle/gen_golden.py attention_fixtures)."""
    g = load_golden("c1_" + case)
    a = load_golden("c1_attn_" + case)
    m = hashed_model(C1, seed=1)
    po = []
    with torch.no_grad():
        R.model_forward(m.state_dict(), m.config, **batch_of(g), probs_out=po)
    L = g["input_ids"].shape[1]
    for i, (local, glob) in enumerate(po):
        assert errs(local[:, :, :L], a[f"a{i}"])["max"] <= 1e-6
        assert errs(glob.transpose(2, 3), a[f"g{i}"])["max"] <= 1e-6


def test_head_at_10k_items_matches_reference():
    """The restated scoring head (cosine / temp + CrossEntropy) against the reference's own
    RecformerForSeqRec head on a 10,000-item frozen catalog (tests/golden/c3_head.npz,
    oracle/gen_golden_head.py): full and sampled softmax, loss and dL/dz."""
    from recformer_amd.hashinit import hash_tensor
    g = load_golden("c3_head")
    items = hash_tensor("catalog", (10000, 768), "weight", seed=4, std=1.0)
    z0 = hash_tensor("pooled", (16, 768), "weight", seed=9, std=1.0)
    for kind in ("full", "sampled"):
        z = z0.clone().requires_grad_(True)
        if kind == "full":
            loss = R.seqrec_loss(R.cosine_scores(z, items, 0.05), g["labels"].long())
        else:
            cand = g["candidates"].long()
            loss = R.seqrec_loss(R.cosine_scores(z, items[cand], 0.05), torch.zeros(16, dtype=torch.long))
        loss.backward()
        assert abs(float(loss) - float(g["loss_" + kind])) <= 1e-5
        assert errs(z.grad, g["dz_" + kind])["max"] <= 1e-7
