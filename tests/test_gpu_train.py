"""Training path (recformer_amd/train.py): losses and every parameter gradient of the HIP
model against autograd through the CPU oracle (oracle/restatement.py, itself pinned to the
reference's forward by tests/test_oracle_golden.py). Dropout off (the reference's dropout RNG
cannot be matched); model.train() otherwise.

Tolerances: fp32 — loss 1e-4 abs, gradients max-abs <= 2e-3 x max|g_ref| per parameter;
autocast bf16 — loss 1e-2 rel, gradient cosine >= 0.99 per parameter (>= 0.95 for tiny
gradients of LayerNorm / bias vectors below 1e-3 of the largest gradient).
"""
import contextlib

import pytest
import torch

from oracle import restatement as R
from recformer_amd import RecformerForSeqRec
from tests.common import C1, batch_of, hashed_model, load_golden

pytestmark = pytest.mark.gpu
CFG = dict(C1, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def _oracle_grads(sd0, cfg, batch, items, labels, temp):
    sd = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in sd0.items()}
    _, p = R.model_forward(sd, cfg, **batch)
    loss = R.seqrec_loss(R.cosine_scores(p, items, temp), labels)
    loss.backward()
    return float(loss.detach()), {k: v.grad for k, v in sd.items() if v.grad is not None}


@pytest.mark.parametrize("mode", ["fp32", "autocast"])
@pytest.mark.parametrize("name", ["c1_full", "c1_ragged"])
def test_seqrec_full_softmax_grads(dev, mode, name):
    g = load_golden(name)
    batch = batch_of(g)
    torch.manual_seed(0)
    items = torch.randn(40, CFG["hidden_size"]) * 0.5
    labels = torch.tensor([3, 17, 0, 39])
    lf = hashed_model(CFG, seed=1)
    ref_loss, ref_g = _oracle_grads(lf.state_dict(), lf.config, batch, items, labels, lf.config.temp)

    model = RecformerForSeqRec(lf.config)
    model.longformer.load_state_dict(lf.state_dict())
    model.config.finetune_negative_sample_size = 0
    model.init_item_embedding(items.clone())
    model = model.to(dev).train()
    ctx = torch.autocast("cuda", dtype=torch.bfloat16) if mode == "autocast" else contextlib.nullcontext()
    with ctx:
        loss = model(**{k: v.to(dev) for k, v in batch.items()}, labels=labels.to(dev))
    loss.backward()
    if mode == "fp32":
        assert abs(float(loss) - ref_loss) <= 1e-4, (float(loss), ref_loss)
    else:
        assert abs(float(loss) - ref_loss) <= 1e-2 * max(1.0, abs(ref_loss))
    gmax = max(float(v.abs().max()) for v in ref_g.values())
    for k, p in model.longformer.named_parameters():
        gr = ref_g[k]
        assert p.grad is not None, k
        gg = p.grad.detach().float().cpu()
        if mode == "fp32":
            err = float((gg - gr).abs().max())
            assert err <= 2e-3 * max(float(gr.abs().max()), 1e-6), (k, err, float(gr.abs().max()))
        else:
            cos = torch.nn.functional.cosine_similarity(gg.reshape(1, -1), gr.reshape(1, -1)).item()
            lim = 0.99 if float(gr.abs().max()) > 1e-3 * gmax else 0.95
            assert cos >= lim or float(gr.abs().max()) < 1e-6, (k, cos)


def test_pretrain_training_step(dev):
    """A10 training: forward + backward + an optimizer step on the pretraining losses."""
    from tests.common import hashed_pretrain, pretrain_inputs
    g = load_golden("c1_pretrain")
    m = hashed_pretrain(CFG).to(dev).train()
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    out = m(**kw)
    # with dropout off the loss equals the reference's eval-mode loss on these inputs
    assert abs(float(out.loss) - float(g["loss"])) <= 1e-4
    out.loss.backward()
    n = sum(1 for p in m.parameters() if p.grad is not None and torch.isfinite(p.grad).all())
    assert n >= len([p for p in m.parameters()]) - 2  # word/pos rows may be all-zero, but finite
    opt.step()
    out2 = m(**kw)
    assert torch.isfinite(out2.loss)
