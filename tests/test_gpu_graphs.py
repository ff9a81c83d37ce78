"""recformer_amd.graphs.CapturedTrainStep: a finetune training step (RecformerForSeqRec forward,
backward, AdamW; finetune.py:98-137) captured once as a HIP graph and replayed, against the same
steps run eagerly — identical losses and parameters without dropout; with attention-probability
dropout, replay k draws exactly the masks of an eager step whose device step counter is k (the
counter the graph advances), so fresh masks per replay and forward/backward agreement are pinned."""
import pytest
import torch

from recformer_amd import RecformerForSeqRec, _lib, graphs
from recformer_amd.optim import AdamW
from tests.common import C1, batch_of, hashed_model, load_golden

pytestmark = pytest.mark.gpu


def _model(dev, att_p=0.0):
    cfg = dict(C1, hidden_dropout_prob=0.0, attention_probs_dropout_prob=att_p)
    lf = hashed_model(cfg, seed=1)
    m = RecformerForSeqRec(lf.config)
    m.longformer.load_state_dict(lf.state_dict())
    m.config.finetune_negative_sample_size = 0
    torch.manual_seed(0)
    m.init_item_embedding(torch.randn(40, cfg["hidden_size"]) * 0.5)
    return m.to(dev).train()


def _batch(dev):
    g = load_golden("c1_full")
    b = {k: v.to(dev) for k, v in batch_of(g).items()}
    b["labels"] = torch.tensor([3, 17, 0, 39], device=dev)
    return b


def _eager_step(m, opt, batch, dtype):
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=dtype):
        loss = m(**batch)
    loss.backward()
    opt.step()
    return float(loss)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_captured_finetune_step_matches_eager(dev, dtype):
    batch = _batch(dev)
    a, b = _model(dev), _model(dev)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    step = graphs.CapturedTrainStep(a, oa, batch, autocast_dtype=dtype, warmup=2)
    losses = [_eager_step(b, ob, batch, dtype) for _ in range(2)]
    for _ in range(3):
        la = float(step())
        losses.append(_eager_step(b, ob, batch, dtype))
        assert abs(la - losses[-1]) <= 1e-5 * max(1.0, abs(la)), (la, losses[-1])
    assert losses[-1] < losses[0]  # it trains
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n
    assert float(next(iter(oa.state.values()))["step"]) == 5.0


def test_captured_step_dropout_masks_follow_device_counter(dev):
    batch = _batch(dev)
    a, b = _model(dev, att_p=0.1), _model(dev, att_p=0.1)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, capturable=True)
    # warmup (eager, host seeds) then capture (host seeds drawn next, mixed with the counter on every
    # replay): the eager model replays the same CPU-generator draws
    torch.manual_seed(123)
    step = graphs.CapturedTrainStep(a, oa, batch, warmup=1)
    torch.manual_seed(123)
    _eager_step(b, ob, batch, torch.bfloat16)
    st = torch.get_rng_state()
    lib = _lib.load()
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    got, ref = [], []
    for k in (1, 2):
        got.append(float(step()))
        counter.fill_(k)
        torch.set_rng_state(st)
        old = lib.rf_set_seed_source(counter.data_ptr())
        try:
            ref.append(_eager_step(b, ob, batch, torch.bfloat16))
        finally:
            lib.rf_set_seed_source(old)
    assert got == pytest.approx(ref, rel=1e-5), (got, ref)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6)
    # the masks change between replays: step 2 with counter 1 would differ
    m3 = _model(dev, att_p=0.1)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        torch.manual_seed(123)
        counter.fill_(1)
        old = lib.rf_set_seed_source(counter.data_ptr())
        try:
            l1 = float(m3(**batch))
            counter.fill_(2)
            torch.manual_seed(123)
            l2 = float(m3(**batch))
        finally:
            lib.rf_set_seed_source(old)
    assert l1 != l2


def test_captured_step_refuses_more_global_tokens(dev):
    batch = _batch(dev)
    m = _model(dev)
    opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-4, capturable=True)
    step = graphs.CapturedTrainStep(m, opt, batch, warmup=1)
    more = dict(batch)
    gm = batch["global_attention_mask"].clone()
    gm[0, : int(batch["attention_mask"][0].sum())] = 1
    more["global_attention_mask"] = gm
    with pytest.raises(ValueError):
        step(more)
    with pytest.raises(ValueError):
        graphs.CapturedTrainStep(m, torch.optim.SGD(m.parameters(), lr=0.1), batch)


def test_captured_pretrain_step_matches_eager(dev):
    """RecformerForPretraining (two views, MLM on both, contrastive; models.py:382-520) captured:
    the masked-LM head over the fixed-capacity row set (labelled rows first, ignored rows after)
    gives the eager step's loss and parameters."""
    from tests.common import hashed_pretrain, pretrain_inputs
    from tests.test_gpu_train import CFG
    g = load_golden("c1_pretrain")
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    a, b = hashed_pretrain(CFG).to(dev).train(), hashed_pretrain(CFG).to(dev).train()
    oa = AdamW(a.parameters(), lr=1e-3, capturable=True)
    ob = AdamW(b.parameters(), lr=1e-3, capturable=True)
    step = graphs.CapturedTrainStep(a, oa, kw, warmup=1)
    assert step.mlm_cap is not None

    def eager():
        ob.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = b(**kw)
        out.loss.backward()
        ob.step()
        return float(out.loss)

    eager()
    for _ in range(2):
        la, lb = float(step()), eager()
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n
