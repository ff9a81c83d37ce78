"""Training path (recformer_amd/train.py): losses and every parameter gradient of the HIP
model against autograd through the CPU oracle (oracle/restatement.py, itself pinned to the
reference's forward by tests/test_oracle_golden.py). Dropout off (the reference's dropout RNG
cannot be matched); model.train() otherwise.

Tolerances: fp32 — loss 1e-4 abs, gradients max-abs <= 2e-3 x max|g_ref| per parameter;
autocast bf16 — loss 1e-2 rel, gradient cosine >= 0.99 per parameter (>= 0.95 for tiny
gradients of LayerNorm / bias vectors below 1e-3 of the largest gradient).
"""
import contextlib
import json
import math
import os
import re

import pytest
import torch
import torch.nn.functional as F

from oracle import restatement as R
from recformer_amd import RecformerForSeqRec, ops
from tests.common import C1, batch_of, hashed_model, load_golden

pytestmark = pytest.mark.gpu
CFG = dict(C1, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def _oracle_grads(sd0, cfg, batch, items, labels, temp):
    sd = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in sd0.items()}
    _, p = R.model_forward(sd, cfg, **batch)
    loss = R.seqrec_loss(R.cosine_scores(p, items, temp), labels)
    loss.backward()
    return float(loss.detach()), {k: v.grad for k, v in sd.items() if v.grad is not None}


@pytest.mark.parametrize("mode", ["fp32", "autocast", "autocast16"])
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
    ctx = (torch.autocast("cuda", dtype=torch.bfloat16 if mode == "autocast" else torch.float16)
           if mode != "fp32" else contextlib.nullcontext())
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


@pytest.mark.parametrize("autocast", [False, True])
def test_pretrain_shared_casts_same_grads(dev, monkeypatch, autocast):
    """The four pretraining passes sharing one autograd cast per weight (models.SHARE_TRAIN_CASTS)
    give the loss and parameter gradients of per-pass casts (dropout off, so both runs are
    deterministic up to the order in which the four passes' gradients are summed)."""
    from recformer_amd import models
    from tests.common import hashed_pretrain, pretrain_inputs
    g = load_golden("c1_pretrain")
    m = hashed_pretrain(CFG).to(dev).train()
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    res = {}
    for share in (False, True):
        monkeypatch.setattr(models, "SHARE_TRAIN_CASTS", share)
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out = m(**kw)
        out.loss.backward()
        res[share] = (float(out.loss), {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-6, abs=1e-6)
    assert res[True][1].keys() == res[False][1].keys()
    for k, ga in res[False][1].items():
        gb = res[True][1][k]
        # under autocast the shared bf16 cast sums the four passes' bf16 weight gradients in
        # bf16 before the fp32 master (as torch autocast's own per-region cast cache does for the
        # reference), per-pass casts sum them in fp32: bf16 rounding of the sum apart
        tol = 1e-5 if not autocast else 1e-2
        assert float((ga - gb).abs().max()) <= tol * max(float(ga.abs().max()), 1e-6), k


@pytest.mark.parametrize("train", [False, True])
def test_pretrain_lm_head_masked_rows_only(dev, monkeypatch, train):
    """The LM head over the labelled rows only (models.LM_HEAD_MASKED_ONLY)
    gives the loss (and, training, the gradients) of the head over every token: the masked-LM
    cross entropy ignores label -100 (models.py:499-510)."""
    from recformer_amd import models
    from tests.common import hashed_pretrain, pretrain_inputs
    g = load_golden("c1_pretrain")
    m = hashed_pretrain(CFG).to(dev).train(train)
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    assert int((kw["mlm_labels_a"] != -100).sum()) > 0
    res = {}
    for masked in (False, True):
        monkeypatch.setattr(models, "LM_HEAD_MASKED_ONLY", masked)
        m.zero_grad(set_to_none=True)
        with torch.set_grad_enabled(train):
            out = m(**kw)
        if train:
            out.loss.backward()
        res[masked] = (float(out.loss), {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-5, abs=1e-6)
    assert abs(res[True][0] - float(g["loss"])) <= 1e-4
    for k, ga in res[False][1].items():
        gb = res[True][1][k]
        assert float((ga - gb).abs().max()) <= 1e-4 * max(float(ga.abs().max()), 1e-6), k


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=2, Lp=256, H=2, lens=[256, 100], globals_=((0, 0), (1, 0))),
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=1, Lp=128, H=1, lens=[128], globals_=()),
    dict(B=2, Lp=1024, H=12, lens=[1024, 700], globals_=((0, 0), (1, 0), (1, 5))),
])
def test_band_attention_bwd_matches_autograd(dev, case, dt):
    """rf_band_attn_bwd (+ the per-sequence reduction of the global-key columns, as
    train._Attention.backward does it) against autograd through the fp32 recompute of the local
    branch (train._local_torch) on the same bf16 inputs; rows with flag != 1 get no gradient.
    Tolerance: max-abs error <= 2e-2 x max |g| (P and dS enter the MFMAs as bf16)."""
    from recformer_amd import ops
    from recformer_amd.train import _global_rows, _local_torch
    from tests.test_gpu_kernels import _attn_case
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 11)
    qkv[:, :D] = (qkv[:, :D].float() * 0.125).to(dt)  # pre-scaled, like the QKV GEMM output
    q, k, v = (qkv[:, i * D:(i + 1) * D] for i in range(3))
    out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32)
    torch.manual_seed(1)
    dout = torch.randn(B * Lp, D, device=dev).to(dt)
    dq, dk, dv, gds, gpr = ops.band_attention_bwd(q, k, v, out, dout, flags, gidx, B, Lp, H)
    if G > 0:
        rows, keep = _global_rows(gidx, B, Lp)
        dkg = torch.einsum("bhig,bihd->bghd", gds[..., :G], q.float().view(B, Lp, H, 64)).reshape(B * G, D)
        dvg = torch.einsum("bhig,bihd->bghd", gpr[..., :G], dout.float().view(B, Lp, H, 64)).reshape(B * G, D)
        dk.index_add_(0, rows[keep], dkg[keep])
        dv.index_add_(0, rows[keep], dvg[keep])
    qr, kr, vr = (t.float().detach().requires_grad_(True) for t in (q, k, v))
    o = _local_torch(qr, kr, vr, flags, gidx, B, Lp, H, 32)
    dmask = (flags.reshape(-1) == 1).float()[:, None]
    ref = torch.autograd.grad(o, (qr, kr, vr), dout.float() * dmask)
    for name, got, r in zip("qkv", (dq, dk, dv), ref):
        err = float((got - r).abs().max())
        assert err <= 2e-2 * max(float(r.abs().max()), 1e-6), (name, err, float(r.abs().max()))


def test_band_attention_bwd_bf16_grads(dev):
    """rf_band_attn_bwd_dt with bf16 gradients (the training path's dqkv) is the fp32 result
    rounded to bf16, bit for bit; the workspace outputs are unchanged."""
    from recformer_amd import ops
    from tests.test_gpu_kernels import _attn_case
    B, Lp, H = 2, 1024, 12
    D = H * 64
    qkv, _, flags, gidx, G = _attn_case(dev, torch.bfloat16, B, Lp, H, [1024, 700], ((0, 0), (1, 0), (1, 5)), 11)
    q, k, v = (qkv[:, i * D:(i + 1) * D] for i in range(3))
    out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32)
    torch.manual_seed(2)
    dout = torch.randn(B * Lp, D, device=dev).to(torch.bfloat16)
    r32 = ops.band_attention_bwd(q, k, v, out, dout, flags, gidx, B, Lp, H,
                                 dqkv=torch.empty(B * Lp, 3 * D, device=dev))
    d16 = torch.empty(B * Lp, 3 * D, device=dev, dtype=torch.bfloat16)
    r16 = ops.band_attention_bwd(q, k, v, out, dout, flags, gidx, B, Lp, H, dqkv=d16)
    for a, b in zip(r32[:3], r16[:3]):
        assert b.dtype == torch.bfloat16
        assert torch.equal(a.to(torch.bfloat16), b)
    assert torch.equal(r32[3], r16[3]) and torch.equal(r32[4], r16[4])


_DROP_CASES = [
    dict(B=2, Lp=256, H=2, lens=[256, 100], globals_=((0, 0), (1, 0))),
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=2, Lp=1024, H=12, lens=[1024, 700], globals_=((0, 0), (1, 0), (1, 5))),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", _DROP_CASES)
def test_band_attention_dropout_fwd(dev, dt, case):
    """Attention-probability dropout (TF:585-586) in the band kernels (rf_band_attn_fwd_drop:
    bf16 pipelined MFMA kernel, fp32 VALU kernel) against the fp32 recompute with the same
    counter-hash mask (train._local_torch, recformer_amd/dropout.py); same seed = same output,
    another seed = another mask; p = 0 is the plain kernel."""
    from recformer_amd.train import _local_torch
    from tests.test_gpu_kernels import _attn_case
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 21)
    q, k, v = (qkv[:, i * D:(i + 1) * D] for i in range(3))
    p, seed = 0.1, 987654321
    out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32, p_drop=p, seed=seed)
    ref = _local_torch(q.float(), k.float(), v.float(), flags, gidx, B, Lp, H, 32, drop=(p, seed))
    local = (flags.reshape(-1) == 1)
    err = float((out.float() - ref)[local].abs().max())
    assert err <= (1e-4 if dt == torch.float32 else 4e-2), err
    assert torch.equal(out, ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32, p_drop=p, seed=seed))
    other = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32, p_drop=p, seed=seed + 1)
    assert not torch.equal(out, other)
    assert torch.equal(ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32, p_drop=0.0, seed=seed),
                       ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32))
    assert float(out.float()[merged.view(-1).to(dev) == 0].abs().max() if (merged == 0).any() else 0.0) == 0.0


@pytest.mark.parametrize("case", _DROP_CASES)
def test_band_attention_dropout_bwd(dev, case):
    """rf_band_attn_bwd_drop (mask regenerated from the seed) against autograd through the fp32
    recompute with the same mask; global-key columns reduced as train._Attention does."""
    from recformer_amd.train import _global_rows, _local_torch
    from tests.test_gpu_kernels import _attn_case
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, torch.bfloat16, B, Lp, H, case["lens"], case["globals_"], 23)
    qkv[:, :D] = (qkv[:, :D].float() * 0.125).to(torch.bfloat16)
    q, k, v = (qkv[:, i * D:(i + 1) * D] for i in range(3))
    p, seed = 0.1, 42
    out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32, p_drop=p, seed=seed)
    torch.manual_seed(3)
    dout = torch.randn(B * Lp, D, device=dev).to(torch.bfloat16)
    dq, dk, dv, gds, gpr = ops.band_attention_bwd(q, k, v, out, dout, flags, gidx, B, Lp, H, p_drop=p, seed=seed)
    if G > 0:
        rows, keep = _global_rows(gidx, B, Lp)
        dkg = torch.einsum("bhig,bihd->bghd", gds[..., :G], q.float().view(B, Lp, H, 64)).reshape(B * G, D)
        dvg = torch.einsum("bhig,bihd->bghd", gpr[..., :G], dout.float().view(B, Lp, H, 64)).reshape(B * G, D)
        dk.index_add_(0, rows[keep], dkg[keep])
        dv.index_add_(0, rows[keep], dvg[keep])
    qr, kr, vr = (t.float().detach().requires_grad_(True) for t in (q, k, v))
    o = _local_torch(qr, kr, vr, flags, gidx, B, Lp, H, 32, drop=(p, seed))
    dmask = (flags.reshape(-1) == 1).float()[:, None]
    ref = torch.autograd.grad(o, (qr, kr, vr), dout.float() * dmask)
    for name, got, r in zip("qkv", (dq, dk, dv), ref):
        err = float((got - r).abs().max())
        assert err <= 2e-2 * max(float(r.abs().max()), 1e-6), (name, err, float(r.abs().max()))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", _DROP_CASES)
def test_global_fold_dropout(dev, dt, case):
    """Global query rows under attention-probability dropout (TF:1036-1037) on the fold kernels
    (rf_global_attn_fold_fwd_drop) against the fp32 torch fold with the same mask
    (train._global_torch); the mask kernel (rf_attn_global_keep) equals train._global_keep
    bit for bit; p = 0 is the plain fold."""
    from recformer_amd.train import _global_keep, _global_torch
    from tests.test_gpu_kernels import _attn_case, _rand
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    _, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=40)
    wkg = _rand((D, D), dev, dt, 0.05, seed=41)
    wvg = _rand((D, D), dev, dt, 0.05, seed=42)
    bkg = _rand((D,), dev, torch.float32, 0.1, seed=43)
    bvg = _rand((D,), dev, torch.float32, 0.5, seed=44)
    qg = _rand((B * G, D), dev, dt, 1.0, seed=45)
    p, seed = 0.1, 20241016
    z = ops.attn_global_keep(gidx, B, Lp, H, p, seed)
    assert torch.equal(z, _global_keep(gidx, B, Lp, H, p, seed))
    kept = float((z > 0).float().mean())
    assert abs(kept - 0.9) < 0.02, kept
    ctx = torch.zeros(B * Lp, D, dtype=dt, device=dev)
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx, p_drop=p, seed=seed)
    ref = _global_torch(qg, h, wkg, bkg, wvg, bvg, flags, B, Lp, H, z)
    plain = _global_torch(qg, h, wkg, bkg, wvg, bvg, flags, B, Lp, H)
    rows = (torch.arange(B, device=dev)[:, None] * Lp + gidx.clamp(min=0).long()).reshape(-1)
    keep = (gidx >= 0).reshape(-1)
    got = ctx[rows].float()
    err = float((got - ref)[keep].abs().max())
    assert err <= 2e-2, err
    assert float((ref - plain)[keep].abs().max()) > 10 * err  # the mask matters at this tolerance
    ctx0 = torch.zeros_like(ctx)
    ctx1 = torch.zeros_like(ctx)
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx0, p_drop=0.0, seed=seed)
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx1)
    assert torch.equal(ctx0, ctx1)


def _drop_model(dev, p_att, p_hid, seed=1):
    lf = hashed_model(dict(C1, hidden_dropout_prob=p_hid, attention_probs_dropout_prob=p_att), seed=seed)
    model = RecformerForSeqRec(lf.config)
    model.longformer.load_state_dict(lf.state_dict())
    model.config.finetune_negative_sample_size = 0
    torch.manual_seed(0)
    model.init_item_embedding(torch.randn(40, C1["hidden_size"]) * 0.5)
    return model.to(dev).train()


def _step(model, batch, labels, autocast, seed):
    model.zero_grad(set_to_none=True)
    torch.manual_seed(seed)
    ctx = torch.autocast("cuda", dtype=torch.bfloat16) if autocast else contextlib.nullcontext()
    with ctx:
        loss = model(**batch, labels=labels)
    loss.backward()
    return float(loss), {k: p.grad.detach().float().clone() for k, p in model.longformer.named_parameters()
                         if p.grad is not None}


@pytest.mark.parametrize("name", ["c1_full", "c1_ragged"])
def test_seqrec_training_with_attention_dropout(dev, name):
    """The reference's training configuration (longformer-base dropouts: attention_probs 0.1,
    hidden 0.1; finetune.py:98-137 under autocast) trains on the HIP path: finite loss and
    gradients, deterministic for a fixed torch seed, a different loss for another seed and
    without dropout. The HIP backward with the regenerated masks (bf16, rf_band_attn_bwd_drop +
    the global rows' closed form) agrees with the fp32 path's recompute through autograd with
    the same masks (attention dropout only: the hidden-dropout masks of the two paths differ):
    gradient cosine >= 0.99 per parameter."""
    g = load_golden(name)
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    labels = torch.tensor([3, 17, 0, 39], device=dev)
    m = _drop_model(dev, 0.1, 0.1)
    l1, g1 = _step(m, batch, labels, True, 11)
    l1b, g1b = _step(m, batch, labels, True, 11)
    l2, _ = _step(m, batch, labels, True, 12)
    assert math.isfinite(l1) and all(torch.isfinite(x).all() for x in g1.values())
    # same seed, same masks: the same loss; gradients equal up to the order of atomic adds (the
    # embedding tables' index_add_)
    assert l1 == l1b
    for k in g1:
        assert float((g1[k] - g1b[k]).abs().max()) <= 1e-5 * max(float(g1[k].abs().max()), 1e-6), k
    assert l1 != l2
    m0 = _drop_model(dev, 0.0, 0.0)
    l0, _ = _step(m0, batch, labels, True, 11)
    assert l0 != l1
    # attention dropout only: bf16 HIP backward vs the fp32 recompute with the same masks
    ma = _drop_model(dev, 0.1, 0.0)
    la, ga = _step(ma, batch, labels, True, 7)
    lf, gf = _step(ma, batch, labels, False, 7)
    assert abs(la - lf) <= 2e-2 * max(1.0, abs(lf))
    gmax = max(float(v.abs().max()) for v in gf.values())
    for k, r in gf.items():
        cos = F.cosine_similarity(ga[k].reshape(1, -1), r.reshape(1, -1)).item()
        lim = 0.99 if float(r.abs().max()) > 1e-3 * gmax else 0.95
        assert cos >= lim or float(r.abs().max()) < 1e-6, (k, cos)


def test_train_mode_under_no_grad_applies_dropout(dev):
    """nn.Dropout applies in train mode whatever the grad mode: model.train() under torch.no_grad()
    draws the same masks (same torch seed) as the gradient-enabled forward — identical loss — and
    differs from eval mode; eval mode under no_grad is the deterministic inference path."""
    g = load_golden("c1_full")
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    labels = torch.tensor([3, 17, 0, 39], device=dev)
    m = _drop_model(dev, 0.1, 0.1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        torch.manual_seed(5)
        l_grad = float(m(**batch, labels=labels))
        torch.manual_seed(5)
        with torch.no_grad():
            l_nograd = float(m(**batch, labels=labels))
        m.eval()
        with torch.no_grad():
            l_eval = float(m(**batch, labels=labels))
            l_eval2 = float(m(**batch, labels=labels))
    assert l_nograd == pytest.approx(l_grad, rel=1e-5, abs=1e-5)
    assert l_eval == l_eval2 and abs(l_eval - l_grad) > 1e-4


def _c2_model(dev):
    from recformer_amd import RecformerConfig
    from recformer_amd.hashinit import hash_init_, hash_tensor
    from tests.common import BASE
    cfg = RecformerConfig(**dict(BASE, item_num=1000, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0))
    model = RecformerForSeqRec(cfg)
    hash_init_(model.longformer, seed=2)
    model.init_item_embedding(hash_tensor("catalog", (1000, 768), "weight", seed=3, std=1.0))
    model.config.finetune_negative_sample_size = 0
    return model.to(dev).train()


# autocast parity contract for the training backward: per parameter group, the HIP gradient's error
# against the reference's fp32 gradient is at most this multiple of the reference's own autocast drift
DRIFT_MULT = 2.0


def _c2_check(model, loss, dz, mode, gz, dev, gscale=1.0):
    """The C2 finetune gradients (times gscale) against tests/golden/c2_grads.npz."""
    ref_loss = float(gz["loss"])
    dz_ref = torch.from_numpy(gz["dz"])
    if mode == "fp32":
        assert abs(float(loss) - ref_loss) <= 1e-3, (float(loss), ref_loss)
        assert float((dz - dz_ref).abs().max()) <= 2e-3 * float(dz_ref.abs().max())
    params = dict(model.longformer.named_parameters())
    gmax = max(float(gz[f"g:{n}:maxabs"]) for n in gz["names"])
    checked = zero = 0
    groups = {}
    for n in gz["names"]:
        n = str(n)
        p = params[n]
        assert p.grad is not None, n
        gr = p.grad.detach().double().flatten() * gscale
        assert bool(torch.isfinite(gr).all()), n
        pos = torch.from_numpy(gz[f"g:{n}:pos"]).to(dev)
        got = gr[pos].float().cpu()
        ref = torch.from_numpy(gz[f"g:{n}:val"])
        mref, nref = float(gz[f"g:{n}:maxabs"]), float(gz[f"g:{n}:norm"])
        if mref < 1e-6 * gmax:
            # mathematically zero, rounding noise in the reference: the key / key_global biases (a
            # softmax-row shift) and the last layer's local q/k/v (only the global CLS row is read)
            assert float(gr.abs().max()) <= 1e-5 * gmax, n
            zero += 1
            continue
        nrm = float(gr.norm())
        if mode == "fp32":
            assert float((got - ref).abs().max()) <= 2e-3 * mref, (n, float((got - ref).abs().max()), mref)
            assert abs(nrm - nref) <= 1e-3 * nref, (n, nrm, nref)
        else:
            # per parameter group (the same tensor across the 12 layers): the HIP autocast gradient's
            # relative L2 error against the reference's fp32 gradient, on the fixture's slices, is held to
            # DRIFT_MULT x the reference's OWN autocast drift on the same slices (its backward under CPU
            # torch.autocast in the same 16-bit type, oracle/gen_golden_grads.py)
            tag = "bf16" if mode == "autocast" else "fp16"
            key = re.sub(r"layer\.\d+\.", "layer.*.", n)
            grp = groups.setdefault(key, [[], [], []])
            grp[0].append(got)
            grp[1].append(ref)
            grp[2].append(torch.from_numpy(gz[f"ac_{tag}:g:{n}:val"]))
        checked += 1
    assert checked + zero == len(gz["names"]) == 270 and zero == 29
    if mode != "fp32":
        rows = []
        for key, (got, ref, rac) in groups.items():
            got, ref, rac = torch.cat(got).double(), torch.cat(ref).double(), torch.cat(rac).double()
            e_hip = float((got - ref).norm() / ref.norm())
            e_ref = float((rac - ref).norm() / ref.norm())
            rows.append({"group": key, "hip_rel_err": e_hip, "ref_autocast_drift": e_ref, "ratio": e_hip / e_ref})
        tag = "bf16" if mode == "autocast" else "fp16"
        dz_ac = torch.from_numpy(gz[f"ac_{tag}:dz"])
        # the loss and dL/dz (the scoring head's input gradient) to the same contract; a floor of 1e-5 relative
        # keeps a single scalar whose reference drift happens to be ~0 from failing on rounding
        for name, e_hip, e_ref in (
                ("loss", abs(float(loss) - ref_loss) / abs(ref_loss),
                 abs(float(gz[f"ac_{tag}:loss"]) - ref_loss) / abs(ref_loss)),
                ("dL/dz", float((dz - dz_ref).norm() / dz_ref.norm()), float((dz_ac - dz_ref).norm() / dz_ref.norm()))):
            rows.append({"group": name, "hip_rel_err": e_hip, "ref_autocast_drift": e_ref,
                         "ratio": e_hip / max(e_ref, 1e-5)})
        os.makedirs(os.path.join("gpurun_out", "drift"), exist_ok=True)
        with open(os.path.join("gpurun_out", "drift", f"c2_grads_{mode}.json"), "w") as f:
            json.dump(rows, f, indent=1)
        bad = [r for r in rows if r.get("ratio", 0.0) > DRIFT_MULT]
        assert not bad, bad


def _c2_fixtures():
    import numpy as np
    gz = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c2_grads.npz"))
    return gz, load_golden("c2_12l")


@pytest.mark.parametrize("mode", ["fp32", "autocast", "autocast16"])
def test_c2_finetune_grads_match_reference(dev, mode):
    """C3 at full model size: RecformerForSeqRec fwd + bwd at 12L/768d, L=1024, B=2 (ragged
    lengths 1024 / 700) on the HIP training path against the REAL reference's gradients
    (tests/golden/c2_grads.npz, oracle/gen_golden_grads.py: models.py full-softmax loss, dropout 0,
    train mode). Per parameter: 256 gradient entries at fixed positions, the L2 norm and max-abs.
    fp32: loss 1e-3 abs, dL/dz and every slice within 2e-3 x max|g| of the parameter, norms 1e-3
    relative. autocast bf16 / fp16 (the reference drivers' mixed precision, finetune.py:106-110): per
    parameter group, and for the loss and dL/dz, the HIP error against the reference's fp32 gradient is
    at most DRIFT_MULT (2) x the reference's OWN autocast drift in the same 16-bit type on the same
    entries (c2_grads.npz ac_bf16 / ac_fp16: its backward under CPU torch.autocast). Measured (round 6):
    ratios 0.07-1.56 (bf16), 0.10-1.36 (fp16); the per-group table goes to gpurun_out/drift/."""
    gz, g12 = _c2_fixtures()
    model = _c2_model(dev)
    keep = {}

    def hook(_m, _i, out):
        out.pooler_output.retain_grad()
        keep["z"] = out.pooler_output

    hdl = model.longformer.register_forward_hook(hook)
    batch = {k: v.to(dev) for k, v in batch_of(g12).items()}
    labels = torch.from_numpy(gz["labels"]).to(dev)
    ctx = (torch.autocast("cuda", dtype=torch.bfloat16 if mode == "autocast" else torch.float16)
           if mode != "fp32" else contextlib.nullcontext())
    with ctx:
        loss = model(**batch, labels=labels)
    loss.backward()
    hdl.remove()
    _c2_check(model, loss, keep["z"].grad.float().cpu(), mode, gz, dev)


def test_c2_finetune_fp16_gradscaler_step(dev):
    """finetune.py:98-137 with --fp16 exactly: torch.cuda.amp.autocast() (fp16), loss divided by the
    8 gradient-accumulation steps, GradScaler() at its initial scale 2^16, scaler.scale(loss).backward(),
    then unscale_ + step + update. The scaled fp16 backward must not overflow where the reference's
    does not: no inf/nan found, the optimizer step runs and the scale is unchanged after update(); the
    unscaled gradients x 8 match the reference's (c2_grads.npz) at the autocast-fp16 tolerances."""
    gz, g12 = _c2_fixtures()
    model = _c2_model(dev)
    keep = {}

    def hook(_m, _i, out):
        out.pooler_output.retain_grad()
        keep["z"] = out.pooler_output

    hdl = model.longformer.register_forward_hook(hook)
    batch = {k: v.to(dev) for k, v in batch_of(g12).items()}
    labels = torch.from_numpy(gz["labels"]).to(dev)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=0.0)
    scaler = torch.amp.GradScaler("cuda")
    assert scaler.get_scale() == 2.0 ** 16
    with torch.autocast("cuda", dtype=torch.float16):
        loss = model(**batch, labels=labels)
    loss8 = loss / 8
    scaler.scale(loss8).backward()
    hdl.remove()
    scaler.unscale_(opt)
    found = sum(float(v.item()) for v in scaler._found_inf_per_device(opt).values())
    assert found == 0.0, "inf/nan in the scaled fp16 gradients"
    before = scaler.get_scale()
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() == before == 2.0 ** 16  # optimizer_was_run (finetune.py:124-127)
    # dL/dz of the retained (fp32) pooler output carries the scale: unscale it for the check
    dz = keep["z"].grad.float().cpu() * 8 / before
    _c2_check(model, loss, dz, "autocast16", gz, dev, gscale=8.0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N", [1000, 50265])
def test_cross_entropy_bwd(dev, dt, N):
    """rf_cross_entropy_bwd = autograd of F.cross_entropy (mean over non-ignored rows, fp32 math) on
    the same logits, scaled by an upstream gradient held on the device; ignored rows are zero."""
    from recformer_amd import ops
    torch.manual_seed(N)
    M = 29
    x = (torch.randn(M, N, device=dev) * 3).to(dt)
    lab = torch.randint(0, N, (M,), device=dev)
    lab[::4] = -100
    xr = x.float().requires_grad_(True)
    loss = F.cross_entropy(xr, lab, ignore_index=-100)
    (gr,) = torch.autograd.grad(loss * 1.7, xr)
    n = (lab != -100).sum().float()
    got = ops.cross_entropy_bwd(x, lab, (torch.tensor(1.7, device=dev) / n).reshape(1))
    assert got.dtype == dt and got.shape == x.shape
    tol = 1e-6 if dt == torch.float32 else 4e-3 * float(gr.abs().max())
    assert float((got.float() - gr).abs().max()) <= tol
    assert float(got[::4].float().abs().max()) == 0.0


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_pretrain_decoder_ce_hip_matches_torch(dev, monkeypatch, dt):
    """Pretraining under autocast with the whole LM head on the HIP kernels — dense + GELU +
    LayerNorm (models.LM_HEAD_HIP, train._LMHeadTransform) and the decoder + masked-LM CE
    (models.DECODER_CE_HIP, train._DecoderCE) — gives the loss and gradients of the torch ops
    (F.linear / F.gelu / F.layer_norm under autocast + F.cross_entropy): loss within 1e-3, gradient
    cosine >= 0.999 for every parameter, the LM head's included."""
    from recformer_amd import models
    from tests.common import hashed_pretrain, pretrain_inputs
    g = load_golden("c1_pretrain")
    m = hashed_pretrain(CFG).to(dev).train()
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    res = {}
    for hip in (False, True):
        monkeypatch.setattr(models, "DECODER_CE_HIP", hip)
        monkeypatch.setattr(models, "LM_HEAD_HIP", hip)
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=dt):
            out = m(**kw)
        out.loss.backward()
        res[hip] = (float(out.loss), {k: p.grad.float().clone() for k, p in m.named_parameters() if p.grad is not None})
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-3, abs=1e-3)
    assert res[True][1].keys() == res[False][1].keys()
    gmax = max(float(v.abs().max()) for v in res[False][1].values())
    for k, ga in res[False][1].items():
        gb = res[True][1][k]
        # key biases: the softmax cancels them, their gradient is rounding noise in both runs
        if float(ga.abs().max()) < 1e-3 * gmax:
            continue
        cos = F.cosine_similarity(ga.reshape(1, -1), gb.reshape(1, -1)).item()
        assert cos >= 0.999, (k, cos)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=3, Lp=1024, H=12, lens=[1024, 700, 129], gpos=[[0], [0], [5]], p=0.0),
    dict(B=2, Lp=256, H=2, lens=[256, 100], gpos=[[0, 77], [3, -1]], p=0.0),
    dict(B=2, Lp=512, H=12, lens=[512, 300], gpos=[[0], [0]], p=0.1),
    dict(B=4, Lp=192, H=6, lens=[192, 64, 190, 1], gpos=[[0, 1, 100, -1], [0, 2, -1, -1], [5, -1, -1, -1], [0, -1, -1, -1]], p=0.1),
])
def test_global_fold_bwd_matches_closed_form(dev, dt, case):
    """rf_global_fold_bwd (the global rows' backward in one pass over h from the forward's fold
    workspace, train._global_bwd_hip) against the closed-form torch backward (train._global_bwd,
    fp32, pinned to autograd by tests/test_train_host.py): dq, dh, dWkg, dWvg, dbvg, with ragged
    lengths, several / empty global slots per sequence and attention dropout (the forward's mask)."""
    from recformer_amd import train as T
    B, Lp, H, p = case["B"], case["Lp"], case["H"], case["p"]
    D = 64 * H
    G = len(case["gpos"][0])
    g = torch.Generator(device="cpu").manual_seed(B * Lp + H)
    flags = torch.zeros(B, Lp, dtype=torch.uint8)
    gidx = torch.full((B, G), -1, dtype=torch.int32)
    for b in range(B):
        flags[b, :case["lens"][b]] = 1
        for k, q in enumerate(case["gpos"][b]):
            if q >= 0:
                flags[b, q] = 2
                gidx[b, k] = q
    flags, gidx = flags.to(dev), gidx.to(dev)
    h = (torch.randn(B * Lp, D, generator=g)).to(dev).to(dt)
    qg = (torch.randn(B * G, D, generator=g) * 0.125).to(dev).to(dt)
    wkg, wvg = ((torch.randn(D, D, generator=g) * 0.05).to(dev).to(dt) for _ in range(2))
    bkg, bvg = ((torch.randn(D, generator=g) * 0.1).to(dev) for _ in range(2))
    out = torch.zeros(B * Lp, D, dtype=dt, device=dev)
    ws = ops.global_fold_workspace(h, B, Lp, H, G)
    seed = 1234
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, out, p_drop=p, seed=seed, ws=ws)
    keep = (gidx >= 0).reshape(-1, 1).float()
    d16 = torch.randn(B * Lp, D, generator=g).to(dev).to(dt)  # the attention output gradient
    rows = (torch.arange(B, device=dev)[:, None] * Lp + gidx.clamp(min=0).long()).reshape(-1)
    gout = d16[rows].float() * keep
    gz = ops.attn_global_keep(gidx, B, Lp, H, p, seed) if p > 0 else None
    ref = T._global_bwd(qg, h, wkg, wvg, flags, B, Lp, H, gout, gz, bvg)
    # rf_global_fold_bwd_full (train._global_bwd_hip) and rf_global_fold_bwd with dw / c given
    got_full = T._global_bwd_hip(qg, h, wkg, wvg, bvg, flags, gidx, B, Lp, H, d16, ws, p, seed)
    got_part = _global_bwd_given_dw(qg, h, wkg, wvg, bvg, flags, gidx, B, Lp, H, gout, ws, p, seed)
    for got in (got_full, got_part):
        for name, a, r in zip(("dq", "dh", "dwkg", "dbkg", "dwvg", "dbvg"), got, ref):
            a, r = a.float(), r.float()
            scale = float(r.abs().max())
            if scale == 0.0:
                assert float(a.abs().max()) == 0.0, name
                continue
            err = float((a - r).abs().max())
            assert err <= 2e-2 * scale, (name, err, scale)
            cos = F.cosine_similarity(a.reshape(1, -1), r.reshape(1, -1)).item()
            assert cos >= 0.9995, (name, cos)


def _global_bwd_given_dw(qg, h, wkg, wvg, bvg, flags, gidx, B, Lp, H, gout, ws, p_drop, seed):
    """rf_global_fold_bwd with dw = Wvg_h^T do_h and c = do_h . bvg_h formed in torch, the per-head
    products with the weights after it in torch (the entry point's documented contract)."""
    D = h.shape[1]
    hd = D // H
    R = gout.shape[0]
    wk = wkg.float().view(H, hd, D)
    wv = wvg.float().view(H, hd, D)
    qH = qg.float().view(R, H, hd).transpose(0, 1)
    doH = gout.float().view(R, H, hd).transpose(0, 1)
    dw = torch.zeros(R, 16, D, dtype=torch.float32, device=h.device)
    dw[:, :H] = torch.bmm(doH, wv).transpose(0, 1)
    cb = None
    if p_drop > 0:
        cb = torch.zeros(R, 16, dtype=torch.float32, device=h.device)
        cb[:, :H] = (doH * bvg.float().view(H, 1, hd)).sum(-1).t()
    dh = torch.empty(B * Lp, D, dtype=h.dtype, device=h.device)
    du, w, stats = ops.global_fold_bwd(h.contiguous(), flags, gidx, B, Lp, H, ws, dw, cb, p_drop, seed, dh)
    duH = du[:, :H].transpose(0, 1)
    dq = torch.bmm(duH, wk.transpose(1, 2)).transpose(0, 1).reshape(R, D)
    dwkg = torch.bmm(qH.transpose(1, 2), duH).reshape(D, D)
    dwvg = torch.bmm(doH.transpose(1, 2), w[:, :H].transpose(0, 1)).reshape(D, D)
    dbvg = (doH * stats[:, :H, 3].t().unsqueeze(-1)).sum(1).reshape(D)
    return dq, dh, dwkg, torch.zeros(D, device=h.device), dwvg, dbvg


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Lp,H,gpos", [(2, 256, 2, [[0, 100], [5, -1]]), (3, 1024, 12, [[0], [0], [-1]]),
                                         (2, 320, 4, [[0, 7, 300, -1], [1, -1, -1, -1]])])
def test_global_kv_grad_matches_torch(dev, dt, B, Lp, H, gpos):
    """rf_global_kv_grad (the global-key / -value rows' gradients added into dk / dv in place) against
    the fp32 einsum of train._global_kv_grad plus the row scatter; empty slots leave dk / dv alone."""
    D = 64 * H
    G = len(gpos[0])
    g = torch.Generator(device="cpu").manual_seed(B + Lp + H)
    gidx = torch.tensor(gpos, dtype=torch.int32, device=dev)
    gds = torch.randn(B, H, Lp, G, generator=g).to(dev)
    gpr = torch.rand(B, H, Lp, G, generator=g).to(dev) / Lp
    q = torch.randn(B * Lp, D, generator=g).to(dev).to(dt)
    d16 = torch.randn(B * Lp, D, generator=g).to(dev).to(dt)
    dqkv = torch.randn(B * Lp, 3 * D, generator=g).to(dev).to(dt)
    dk, dv = dqkv[:, D:2 * D], dqkv[:, 2 * D:]
    ref_k, ref_v = dk.float().clone(), dv.float().clone()
    ek = torch.einsum("bhig,bihd->bghd", gds, q.float().view(B, Lp, H, 64)).reshape(B, G, D)
    ev = torch.einsum("bhig,bihd->bghd", gpr, d16.float().view(B, Lp, H, 64)).reshape(B, G, D)
    for b in range(B):
        for k in range(G):
            if gpos[b][k] >= 0:
                ref_k[b * Lp + gpos[b][k]] += ek[b, k]
                ref_v[b * Lp + gpos[b][k]] += ev[b, k]
    before = dqkv.clone()
    ops.global_kv_grad(gds, gpr, q, d16, gidx, B, Lp, H, dk, dv)
    torch.cuda.synchronize()
    assert torch.equal(dqkv[:, :D], before[:, :D])  # the q columns are untouched
    for got, ref in ((dk, ref_k), (dv, ref_v)):
        err = (got.float() - ref).abs()
        tol = 1e-2 if dt == torch.bfloat16 else 2e-3
        assert float((err / (ref.abs() + 1.0)).max()) <= tol
    untouched = torch.ones(B * Lp, dtype=torch.bool, device=dev)
    for b in range(B):
        for k in range(G):
            if gpos[b][k] >= 0:
                untouched[b * Lp + gpos[b][k]] = False
    assert torch.equal(dqkv[untouched], before[untouched])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_global_query_bwd_matches_torch(dev, dt):
    """rf_global_query_bwd (backward of qg = (h[global rows] Wqg^T + b) * s) against torch in fp32:
    dWqg, dbqg, and the global rows' input gradient added in place into dh (other rows untouched;
    an empty slot contributes nothing)."""
    B, Lp, D, G = 3, 128, 256, 2
    s = 0.125
    g = torch.Generator(device="cpu").manual_seed(5)
    gidx = torch.tensor([[0, 37], [5, -1], [-1, -1]], dtype=torch.int32, device=dev)
    h = torch.randn(B * Lp, D, generator=g).to(dev).to(dt)
    w = (torch.randn(D, D, generator=g) * 0.05).to(dev).to(dt)
    wT = (w.float() * s).to(dt).t().contiguous()
    dqg = torch.randn(B * G, D, generator=g).to(dev)
    dqg[gidx.reshape(-1) < 0] = 0
    dh = torch.randn(B * Lp, D, generator=g).to(dev).to(dt)
    before = dh.clone()
    dwqg, dbqg = ops.global_query_bwd(gidx, dqg, s, h, wT, dh, B, Lp)
    rows = (torch.arange(B, device=dev)[:, None] * Lp + gidx.clamp(min=0).long()).reshape(-1)
    keep = (gidx.reshape(-1) >= 0).float()[:, None]
    dqs = dqg * s * keep
    ref_w = dqs.t() @ h.index_select(0, rows).float()
    assert torch.allclose(dwqg, ref_w, rtol=1e-4, atol=1e-4)
    assert torch.allclose(dbqg, dqs.sum(0), rtol=1e-5, atol=1e-5)
    ref_dh = before.float().index_add(0, rows, (dqg * keep) @ wT.float().t())
    tol = 2e-2 if dt == torch.bfloat16 else 4e-3
    assert float(((dh.float() - ref_dh).abs() / (ref_dh.abs() + 1)).max()) <= tol
    other = torch.ones(B * Lp, dtype=torch.bool, device=dev)
    other[rows[keep[:, 0] > 0]] = False
    assert torch.equal(dh[other], before[other])


@pytest.mark.parametrize("kind", ["full", "sampled"])
def test_hip_head_at_10k_items_matches_reference(dev, kind):
    """The HIP training head (train.cos_scores_train on rf_cos_score_*, rf_cos_score_bwd and
    train.cross_entropy_train on rf_cross_entropy_*) at C3's 10,000-item catalog against the
    reference's own head (tests/golden/c3_head.npz): loss <= 1e-5 abs, dL/dz <= 1e-4 x max|dz|."""
    from recformer_amd import train
    from recformer_amd.hashinit import hash_tensor
    g = load_golden("c3_head")
    table = hash_tensor("catalog", (10000, 768), "weight", seed=4, std=1.0).to(dev).contiguous()
    rnorm = ops.row_inv_norm(table)
    z = hash_tensor("pooled", (16, 768), "weight", seed=9, std=1.0).to(dev).requires_grad_(True)
    if kind == "full":
        loss = train.cross_entropy_train(train.cos_scores_train(z, table, rnorm, 20.0), g["labels"].to(dev))
    else:
        logits = train.cos_scores_train(z, table, rnorm, 20.0, g["candidates"].to(dev).long())
        loss = train.cross_entropy_train(logits, torch.zeros(16, dtype=torch.long, device=dev))
    loss.backward()
    assert abs(float(loss) - float(g["loss_" + kind])) <= 1e-5, (float(loss), float(g["loss_" + kind]))
    ref = g["dz_" + kind]
    err = float((z.grad.cpu() - ref).abs().max())
    assert err <= 1e-4 * float(ref.abs().max()), (err, float(ref.abs().max()))


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_cls_last_layer_training_matches_full(dev, monkeypatch, dtype, p_drop):
    """RecformerForSeqRec training with the last layer on the CLS rows (train._GlobalCLS): the loss and
    every parameter gradient equal the full last layer's — including exact zeros (not None) for the last
    layer's local query / key / value projections, which never reach the CLS rows. With hidden and
    attention dropout on (the reference finetune's 0.1, same torch seed): the compacted CLS rows draw
    the hidden-dropout masks of their full-layer rows b * Lp (mask_row_mul) and the fold the global
    rows' attention masks, so both paths train on the same masks."""
    from recformer_amd import models
    g = load_golden("c1_ragged")
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    labels = torch.tensor([3, 17, 0, 39], device=dev)
    torch.manual_seed(0)
    items = torch.randn(40, CFG["hidden_size"]) * 0.5
    res = {}
    for prune in (False, True):
        monkeypatch.setattr(models, "PRUNE_LAST_LAYER", prune)
        lf = hashed_model(dict(CFG, hidden_dropout_prob=p_drop, attention_probs_dropout_prob=p_drop), seed=1)
        m = RecformerForSeqRec(lf.config)
        m.longformer.load_state_dict(lf.state_dict())
        m.config.finetune_negative_sample_size = 0
        m.init_item_embedding(items.clone())
        m = m.to(dev).train()
        torch.manual_seed(123)  # the pass's dropout seeds
        with torch.autocast("cuda", dtype=dtype):
            loss = m(**batch, labels=labels)
        loss.backward()
        assert m.longformer._last_pruned == prune
        res[prune] = (float(loss), {k: p.grad for k, p in m.longformer.named_parameters()})
    assert abs(res[True][0] - res[False][0]) <= 2e-3 * max(1.0, abs(res[False][0]))
    nl = CFG["num_hidden_layers"]
    gmax = max(float(g.abs().max()) for g in res[False][1].values() if g is not None)
    for k, gf in res[False][1].items():
        gp = res[True][1][k]
        assert gp is not None, k
        if f"layer.{nl - 1}.attention.self." in k and k.split(".")[-2] in ("query", "key", "value"):
            assert not gp.any() and not gf.any(), k
            continue
        if float(gf.abs().max()) < 1e-7:
            continue
        if k.endswith("key.bias") or k.endswith("key_global.bias"):
            # mathematically zero (a key bias shifts every score of a softmax row equally): rounding noise
            # on both paths, so bounded instead of correlated
            assert float(gp.abs().max()) <= 1e-3 * gmax and float(gf.abs().max()) <= 1e-3 * gmax, k
            continue
        cos = F.cosine_similarity(gp.float().reshape(1, -1), gf.float().reshape(1, -1)).item()
        assert cos >= 0.999, (k, cos)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_side_stream_switches_bit_identical(dev, monkeypatch, dtype):
    """The training step's side-stream placements change where kernels run, not what they compute:
    the fold's first stage beside the band attention (train.FOLD_SIDE_TRAIN: stage 1 + stage 2 instead of
    the one-call fold), the global rows' backward on the weight-gradient stream (train.GLOBAL_BWD_SIDE) and
    the Linear weight gradients accumulated on that stream with one join at the end of the backward
    (train.deferred_weight_grads) give bit-identical losses and gradients in each combination, with hidden
    and attention dropout on (a missing stream dependency would show as a sometimes-different gradient)."""
    from recformer_amd import train as T
    g = load_golden("c1_ragged")
    batch = {k: v.to(dev) for k, v in batch_of(g).items()}
    labels = torch.tensor([3, 17, 0, 39], device=dev)
    torch.manual_seed(0)
    items = torch.randn(40, CFG["hidden_size"]) * 0.5
    lf = hashed_model(dict(CFG, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1), seed=1)
    res = {}
    for fold_side, bwd_side, defer in ((True, True, True), (True, True, False), (False, False, True),
                                       (False, False, False), (True, False, True), (False, True, False)):
        monkeypatch.setattr(T, "FOLD_SIDE_TRAIN", fold_side)
        monkeypatch.setattr(T, "GLOBAL_BWD_SIDE", bwd_side)
        m = RecformerForSeqRec(lf.config)
        m.longformer.load_state_dict(lf.state_dict())
        m.config.finetune_negative_sample_size = 0
        m.init_item_embedding(items.clone())
        m = m.to(dev).train()
        for rep in range(2):  # twice: a race would rarely repeat its result
            # rep 1 accumulates onto zeroed (not None) gradients: the deferred path's add_ form
            m.zero_grad(set_to_none=rep == 0)
            torch.manual_seed(321)
            with torch.autocast("cuda", dtype=dtype):
                loss = m(**batch, labels=labels)
            with T.deferred_weight_grads(defer):
                loss.backward()
            torch.cuda.synchronize()
            res[(fold_side, bwd_side, defer, rep)] = (loss.detach().float().cpu(),
                                                      {k: p.grad.detach().clone() for k, p in
                                                       m.longformer.named_parameters() if p.grad is not None})
    ref_loss, ref_g = res[(True, True, True, 0)]
    for key, (loss, grads) in res.items():
        assert torch.equal(loss, ref_loss), key
        assert grads.keys() == ref_g.keys(), key
        for k in ref_g:
            assert torch.equal(grads[k], ref_g[k]), (key, k)
