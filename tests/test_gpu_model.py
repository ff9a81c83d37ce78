"""Tier (iii): end-to-end RecformerModel / RecformerForSeqRec on the HIP path against the
golden fixtures produced by the real reference (and the pinned oracle).

Tolerances (north star + SURVEY.md §8c, where the reference's OWN bf16 autocast drifts
0.008 max-abs at 1 layer and 0.028 at 12):
  fp32: max-abs <= 1e-3 end to end;
  bf16: max-abs <= 1e-2 for a single layer; end to end mean-abs <= 1e-2, rel-L2 <= 1e-2,
        pooler cosine >= 0.9999 and top-10 items of the scores agree.
"""
import pytest
import torch
import torch.nn.functional as F

from recformer_amd import RecformerForSeqRec
from recformer_amd.hashinit import hash_tensor
from tests.common import BASE, C1, batch_of, errs, hashed_model, load_golden

pytestmark = pytest.mark.gpu


def _run(model, g, dev, dt):
    model = model.to(dev)
    if dt == torch.bfloat16:
        model = model.to(torch.bfloat16)
    with torch.no_grad():
        out = model(**{k: v.to(dev) for k, v in batch_of(g).items()})
    return out


@pytest.mark.parametrize("name", ["c1_full", "c1_ragged", "c1_l200"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_c1_golden(dev, name, dt):
    g = load_golden(name)
    out = _run(hashed_model(C1, seed=1), g, dev, dt)
    ref = g["last_hidden_state"]
    assert out.last_hidden_state.shape == ref.shape
    e = errs(out.last_hidden_state, ref)
    if dt == torch.float32:
        assert e["max"] <= 1e-3, e
    else:
        assert e["mean"] <= 1e-2 and e["rel"] <= 1e-2, e
        cos = F.cosine_similarity(out.pooler_output.float().cpu(), g["pooler_output"], dim=-1)
        assert cos.min().item() >= 0.9999, cos


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_one_layer_768(dev, dt):
    g = load_golden("l1_768")
    out = _run(hashed_model(dict(BASE, num_hidden_layers=1, attention_window=[64]), seed=4), g, dev, dt)
    e = errs(out.last_hidden_state, g["last_hidden_state"])
    assert e["max"] <= (1e-3 if dt == torch.float32 else 1e-2), e


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_12l_768_encode_score_losses(dev, dt):
    g = load_golden("c2_12l")
    m = hashed_model(BASE, seed=2, cls=RecformerForSeqRec, item_num=1000)
    items = hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0)
    m.init_item_embedding(items)
    m = m.to(dev)
    if dt == torch.bfloat16:
        m = m.to(torch.bfloat16)
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    with torch.no_grad():
        out = m.longformer(**batch)
        scores = m(**batch)
        loss = m(**batch, labels=g["labels"].to(dev))
        s_cand = m.similarity_score(out.pooler_output, g["candidates"].to(dev))
    ep = errs(out.pooler_output, g["pooler_output"])
    eh = errs(out.last_hidden_state[:, g["rows"]], g["hidden_rows"])
    es = errs(scores, g["scores"])
    if dt == torch.float32:
        assert ep["max"] <= 1e-3 and eh["max"] <= 1e-3, (ep, eh)
        assert es["max"] <= 2e-2, es          # scores are cos/0.05: 1e-3 * 20
        assert abs(loss.item() - g["loss_full"].item()) <= 1e-3
        assert errs(s_cand, g["scores_cand"])["max"] <= 2e-2
    else:
        assert eh["mean"] <= 1e-2 and eh["rel"] <= 1e-2, eh
        cos = F.cosine_similarity(out.pooler_output.float().cpu(), g["pooler_output"], dim=-1)
        assert cos.min().item() >= 0.9999, cos
        top_ours = scores.float().cpu().topk(10, dim=1).indices
        top_ref = g["scores"].topk(10, dim=1).indices
        for b in range(top_ref.shape[0]):
            assert set(top_ours[b].tolist()) == set(top_ref[b].tolist())
        assert abs(loss.item() - g["loss_full"].item()) <= 5e-2


def test_bf16_matches_fp32_path_under_autocast(dev):
    """fp32 parameters + CUDA autocast(bf16) takes the bf16 kernels (finetune.py:107 usage)."""
    g = load_golden("c1_full")
    m = hashed_model(C1, seed=1).to(dev)
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(**batch)
    assert out.last_hidden_state.dtype == torch.bfloat16
    e = errs(out.last_hidden_state, g["last_hidden_state"])
    assert e["mean"] <= 1e-2 and e["rel"] <= 1e-2, e


def test_return_tuple_and_hidden_states(dev):
    g = load_golden("c1_ragged")
    m = hashed_model(C1, seed=1).to(dev)
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    with torch.no_grad():
        t = m(**batch, return_dict=False, output_hidden_states=True)
    assert len(t) == 3 and len(t[2]) == C1["num_hidden_layers"] + 1
    assert errs(t[0], g["last_hidden_state"])["max"] <= 1e-3
    assert torch.equal(t[2][-1], t[0])
