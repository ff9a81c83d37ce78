"""Host-side (CPU) checks of the training path's torch algebra (no GPU needed)."""
import numpy as np
import pytest
import torch

from recformer_amd import train


@pytest.mark.parametrize("merged", [True, False])
@pytest.mark.parametrize("drop", [False, True])
@pytest.mark.parametrize("B,Lp,H,G", [(2, 64, 2, 1), (3, 128, 3, 2), (1, 192, 12, 3)])
def test_global_bwd_closed_form_matches_autograd(B, Lp, H, G, drop, merged, monkeypatch):
    """train._global_bwd (closed-form gradient of the global rows' fold algebra, TF:964-1057)
    against autograd through train._global_torch on the same inputs: ragged valid lengths,
    several global slots, one empty slot (zero query row and zero output gradient); with
    attention-probability dropout (TF:1036-1037: the dropped probabilities also scale the value
    bias) through the kernels' hash mask. merged: the products over h as three batched GEMMs
    (train.GLOBAL_BWD_MERGED) or six."""
    monkeypatch.setattr(train, "GLOBAL_BWD_MERGED", merged)
    g = torch.Generator().manual_seed(B * 100 + Lp + H + G)
    D = 64 * H
    qg = torch.randn(B * G, D, generator=g, dtype=torch.float64)
    h = torch.randn(B * Lp, D, generator=g, dtype=torch.float64)
    wkg = torch.randn(D, D, generator=g, dtype=torch.float64) * 0.05
    bkg = torch.randn(D, generator=g, dtype=torch.float64) * 0.1
    wvg = torch.randn(D, D, generator=g, dtype=torch.float64) * 0.05
    bvg = torch.randn(D, generator=g, dtype=torch.float64) * 0.1
    flags = torch.ones(B, Lp, dtype=torch.uint8)
    for b in range(B):
        n = Lp - 17 * b
        flags[b, n:] = 0
    gout = torch.randn(B * G, D, generator=g, dtype=torch.float64)
    if G > 1:
        qg[G - 1] = 0  # an empty slot of sequence 0
        gout[G - 1] = 0
    z = None
    if drop:
        gidx = torch.stack([torch.arange(G) * 5 for _ in range(B)]).to(torch.int32)
        z = train._global_keep(gidx, B, Lp, H, 0.3, 12345)
        assert 0.55 < float((z > 0).double().mean()) < 0.85
    ins = [t.clone().requires_grad_(True) for t in (qg, h, wkg, bkg, wvg, bvg)]
    og = train._global_torch(*ins, flags, B, Lp, H, z)
    ref = torch.autograd.grad(og, ins, gout.float(), allow_unused=True)
    got = train._global_bwd(qg, h, wkg, wvg, flags, B, Lp, H, gout, z, bvg)
    names = ("dqg", "dh", "dwkg", "dbkg", "dwvg", "dbvg")
    # the key bias only shifts each softmax row: its gradient is zero (autograd: rounding noise)
    assert torch.count_nonzero(got[3]) == 0
    assert ref[3] is None or float(ref[3].abs().max()) <= 1e-4 * float(ref[0].abs().max())
    for name, r, x in zip(names, ref, got):
        if name == "dbkg":
            continue
        r = torch.zeros_like(x) if r is None else r.float()
        scale = max(float(r.abs().max()), 1e-3)
        assert float((x.float() - r).abs().max()) <= 1e-4 * scale, name


def test_weight_grad_split_k_matches_single_gemm():
    """train._weight_grad (split-K batched dW = dC^T A, fp32 partials and result) against the
    product in fp64, within bf16 rounding (on the CPU the partials are bf16 products)."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 16384, 48, 40
    dc = torch.randn(M, N, generator=g).to(torch.bfloat16)
    a = torch.randn(M, K, generator=g).to(torch.bfloat16)
    ref = dc.double().t() @ a.double()
    got = train._weight_grad(dc, a)
    assert got.dtype == torch.float32 and got.shape == (N, K)  # fp32: the master weight's dtype
    assert float((got.double() - ref).abs().max()) <= 2e-2 * float(ref.abs().max())
    # a short reduction stays one GEMM
    assert torch.equal(train._weight_grad(dc[:1024], a[:1024]), (dc[:1024].t() @ a[:1024]).float())


def _drop_keep_np(seed, idx, thresh):
    """rf_common.h drop_keep written with numpy uint32 wrap-around arithmetic."""
    u32 = np.uint32
    with np.errstate(over="ignore"):
        idx = np.asarray(idx, dtype=np.uint64)
        h = (idx & 0xFFFFFFFF).astype(u32) * u32(0x9E3779B1) ^ (idx >> 32).astype(u32) * u32(0x85EBCA77) \
            ^ u32(seed & 0xFFFFFFFF)
        h ^= h >> u32(16)
        h *= u32(0x85EBCA6B)
        h ^= u32((seed >> 32) & 0xFFFFFFFF)
        h ^= h >> u32(13)
        h *= u32(0xC2B2AE35)
        h ^= h >> u32(16)
    return h >= u32(thresh)


@pytest.mark.parametrize("p", [0.1, 0.5, 0.9])
def test_dropout_hash_torch_matches_c(p):
    """recformer_amd.dropout.keep (int64 torch ops) is the kernels' counter hash bit for bit, and
    keeps a 1 - p fraction; thresh / scale are the kernels' fp32-derived values."""
    from recformer_amd import dropout
    thresh, scale = dropout.drop_params(p)
    assert thresh == int(float(np.float32(p)) * 2 ** 32)
    assert scale == float(np.float32(1) / (np.float32(1) - np.float32(p)))
    g = torch.Generator().manual_seed(5)
    idx = torch.cat([torch.randint(0, 2 ** 62, (20000,), generator=g), torch.arange(20000),
                     torch.tensor([2 ** 32 - 1, 2 ** 32, 2 ** 40 + 7])])
    for seed in (0, 1, 2 ** 61 + 12345, 0xDEADBEEFCAFE):
        got = dropout.keep(seed, idx, thresh).numpy()
        ref = _drop_keep_np(seed, idx.numpy(), thresh)
        assert (got == ref).all()
        assert abs(got[:20000].mean() - (1 - p)) < 0.02


def test_global_bwd_bf16_dh_close_to_fp32():
    """dh_dtype=bfloat16 (the 16-bit training modes): dh from bf16 operands with fp32 accumulation
    stays within a few bf16 ulps of the fp32 product rounded to bf16; the other gradients are the
    same fp32 values."""
    g = torch.Generator().manual_seed(7)
    B, Lp, H, G = 2, 128, 4, 2
    D = 64 * H
    qg = torch.randn(B * G, D, generator=g)
    h = torch.randn(B * Lp, D, generator=g)
    wkg = torch.randn(D, D, generator=g) * 0.05
    wvg = torch.randn(D, D, generator=g) * 0.05
    flags = torch.ones(B, Lp, dtype=torch.uint8)
    flags[1, 100:] = 0
    gout = torch.randn(B * G, D, generator=g)
    ref = train._global_bwd(qg, h, wkg, wvg, flags, B, Lp, H, gout)
    got = train._global_bwd(qg, h, wkg, wvg, flags, B, Lp, H, gout, dh_dtype=torch.bfloat16)
    assert got[1].dtype == torch.bfloat16
    err = (got[1].float() - ref[1]).abs().max() / ref[1].abs().max()
    assert err < 1e-2, float(err)  # measured 4.6e-3; bf16 rounding alone 2.2e-3
    for n in (0, 2, 4, 5):
        assert torch.equal(got[n], ref[n])


@pytest.mark.parametrize("G", [1, 3])
def test_global_kv_grad_blockdiag_matches_einsum(G, monkeypatch):
    """train._global_kv_grad: the block-diagonal batched product (no copy of the strided q slice)
    equals the einsum form on the same bf16 operands (fp32 accumulation both ways)."""
    g = torch.Generator().manual_seed(G)
    B, Lp, H = 2, 96, 3
    D = 64 * H
    qkv = torch.randn(B * Lp, 3 * D, generator=g).to(torch.bfloat16)
    q = qkv[:, :D]  # strided column slice, as in _Attention.backward
    w = torch.randn(B, H, Lp, G, generator=g) * 0.1
    monkeypatch.setattr(train, "GLOBAL_KV_BLOCKDIAG", False)
    ref = train._global_kv_grad(w, q, B, Lp, H).float()
    monkeypatch.setattr(train, "GLOBAL_KV_BLOCKDIAG", True)
    got = train._global_kv_grad(w, q, B, Lp, H)
    assert got.shape == (B * G, D) and got.dtype == torch.bfloat16
    exact = (w.double().permute(0, 3, 1, 2).unsqueeze(-1) *
             q.double().view(B, Lp, H, 64).permute(0, 2, 1, 3).unsqueeze(1)).sum(3).reshape(B * G, D)
    scale = float(exact.abs().max())
    assert float((got.double() - exact).abs().max()) <= 1e-2 * scale
    assert float((got.float() - ref).abs().max()) <= 1e-2 * scale
