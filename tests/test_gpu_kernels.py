"""Tier (ii): each HIP kernel (through the C ABI) against an fp32 reference of the same op.

Tolerances: fp32 kernels 1e-4 (exact-f32 MFMA, different summation order); bf16 kernels
are compared against the fp32 op on the SAME bf16-rounded inputs, so the only error is
bf16 output rounding (~2^-9 relative) plus bf16 P in the attention PV product.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import restatement as R
from recformer_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _rand(shape, dev, dt, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dev).to(dt)


def _tol(dt):
    return 1e-4 if dt == torch.float32 else 2e-2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(64, 128, 64), (200, 200, 768), (1024, 768, 768), (320, 3840, 768), (256, 768, 3072)])
@pytest.mark.parametrize("epi", [ops.RF_EPI_NONE, ops.RF_EPI_BIAS, ops.RF_EPI_BIAS_GELU, ops.RF_EPI_BIAS_RESID])
def test_gemm_epilogues(dev, dt, M, N, K, epi):
    a = _rand((M, K), dev, dt, seed=1)
    w = _rand((N, K), dev, dt, 0.05, seed=2)
    b = _rand((N,), dev, torch.float32, seed=3)
    r = _rand((M, N), dev, dt, seed=4)
    sc = (N // 3) // 16 * 16          # head-aligned q columns
    out = ops.gemm(a, w, b if epi else None, epi, resid=r if epi == ops.RF_EPI_BIAS_RESID else None,
                   scale_cols=sc, col_scale=0.125)
    ref = a.float() @ w.float().t()
    if epi:
        ref = ref + b
    ref[:, :sc] *= 0.125
    if epi == ops.RF_EPI_BIAS_GELU:
        ref = F.gelu(ref)
    if epi == ops.RF_EPI_BIAS_RESID:
        ref = ref + r.float()
    err = (out.float() - ref).abs().max().item()
    assert err <= _tol(dt) * max(1.0, ref.abs().max().item()), err


def test_gemm_bf16_fp32_output_and_mixed_layernorm(dev):
    """bf16 GEMM writing the fp32 pre-LN residual sum, then LN fp32 -> bf16."""
    a = _rand((300, 768), dev, torch.bfloat16, seed=11)
    w = _rand((768, 768), dev, torch.bfloat16, 0.05, seed=12)
    b = _rand((768,), dev, torch.float32, seed=13)
    r = _rand((300, 768), dev, torch.bfloat16, seed=14)
    t = ops.gemm(a, w, b, ops.RF_EPI_BIAS_RESID, resid=r, out_f32=True)
    assert t.dtype == torch.float32
    ref = a.float() @ w.float().t() + b + r.float()
    assert (t - ref).abs().max().item() <= 1e-3
    lw = _rand((768,), dev, torch.float32, seed=15)
    lb = _rand((768,), dev, torch.float32, seed=16)
    y, y32 = ops.layernorm(t, lw, lb, 1e-5, out_dtype=torch.bfloat16, want_f32=True)
    assert y.dtype == torch.bfloat16 and y32.dtype == torch.float32
    assert (y32 - F.layer_norm(ref, (768,), lw, lb, 1e-5)).abs().max().item() <= 1e-3
    t2 = ops.gemm(a, w, b, ops.RF_EPI_BIAS_RESID, resid=y32, out_f32=True)
    assert (t2 - (a.float() @ w.float().t() + b + y32)).abs().max().item() <= 1e-3
    yr = F.layer_norm(ref, (768,), lw, lb, 1e-5)
    assert (y.float() - yr).abs().max().item() <= 2 ** -8 * yr.abs().max().item() + 1e-3


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_resid_ln(dev, dt):
    """Residual = LayerNorm(previous pre-LN rows) recomputed in the GEMM epilogue."""
    M, N, K = 300, 768, 768
    a = _rand((M, K), dev, dt, seed=21)
    w = _rand((N, K), dev, dt, 0.05, seed=22)
    b = _rand((N,), dev, torch.float32, seed=23)
    x = _rand((M, N), dev, torch.float32, 2.0, seed=24) + 0.5
    g = _rand((N,), dev, torch.float32, seed=25)
    be = _rand((N,), dev, torch.float32, seed=26)
    y, mean, rstd = ops.layernorm(x, g, be, 1e-5, out_dtype=dt, stats=True)
    out = ops.gemm_resid_ln(a, w, b, x, mean, rstd, g, be)
    ref = a.float() @ w.float().t() + b + F.layer_norm(x, (N,), g, be, 1e-5)
    assert out.dtype == torch.float32
    assert (out - ref).abs().max().item() <= (1e-4 if dt == torch.float32 else 1e-3) * ref.abs().max().item()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_gemm_strided_views(dev, dt):
    """Column slices of a fused buffer as A (the q/k/v views) and as W (packed weights)."""
    big = _rand((256, 5 * 128), dev, dt, seed=5)
    a = big[:, 128:256]
    w = _rand((3 * 64, 128), dev, dt, 0.1, seed=6)[:128]
    out = ops.gemm(a, w, None, ops.RF_EPI_NONE)
    ref = a.float() @ w.float().t()
    assert (out.float() - ref).abs().max().item() <= _tol(dt) * ref.abs().max().item()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [128, 768])
def test_layernorm(dev, dt, D):
    x = _rand((333, D), dev, dt, 3.0, seed=7) + 1.0
    w = _rand((D,), dev, torch.float32, seed=8)
    b = _rand((D,), dev, torch.float32, seed=9)
    y, mean, rstd = ops.layernorm(x, w, b, 1e-5, stats=True)
    ref = F.layer_norm(x.float(), (D,), w, b, 1e-5)
    # bf16: output rounding only (half an ulp = 2^-9 relative)
    tol = 1e-4 if dt == torch.float32 else 2 ** -8 * ref.abs().max().item()
    assert (y.float() - ref).abs().max().item() <= tol
    assert torch.allclose(mean, x.float().mean(1), atol=1e-4)


@pytest.mark.parametrize("D", [128, 768])
@pytest.mark.parametrize("inplace", [False, True])
def test_add_layernorm(dev, D, inplace):
    """LN(bf16 dense + fp32 residual) -> bf16 + fp32 stream (TF:1064-1071 under autocast)."""
    M = 333
    x = _rand((M, D), dev, torch.bfloat16, 3.0, seed=17)
    res = _rand((M, D), dev, torch.float32, 2.0, seed=18) + 0.5
    w = _rand((D,), dev, torch.float32, seed=19)
    b = _rand((D,), dev, torch.float32, seed=20)
    ref = F.layer_norm(x.float() + res, (D,), w, b, 1e-5)
    y, y32 = ops.add_layernorm(x, res, w, b, 1e-5, res_out=res if inplace else None)
    assert (y32 - ref).abs().max().item() <= 1e-4
    assert (y.float() - ref).abs().max().item() <= 2 ** -8 * ref.abs().max().item()
    assert y.dtype == torch.bfloat16 and (y32.data_ptr() == res.data_ptr()) == inplace


def _split_ref(v):
    """Host restatement of rf_common.h split_f32: hi = top half of the fp32 bits rounded
    half-up, lo = the low 16 bits."""
    u = v.float().contiguous().view(torch.int32).long() & 0xFFFFFFFF
    return (((u + 0x8000) >> 16) & 0xFFFF), u & 0xFFFF


@pytest.mark.parametrize("D", [128, 768])
@pytest.mark.parametrize("mode", ["planes", "f32", "both", "nores"])
def test_add_layernorm_split(dev, D, mode):
    """LN(bf16 dense + fp32 stream) on the split stream, vs the fp32 torch LayerNorm of the
    decoded stream: the planes decode exactly to the fp32 output (when both are written) and
    the hi plane is that value rounded half-up to bf16 (within half a bf16 ulp); in place."""
    M = 333
    x = _rand((M, D), dev, torch.bfloat16, 3.0, seed=17)
    res = _rand((M, D), dev, torch.float32, 2.0, seed=18) + 0.5
    w = _rand((D,), dev, torch.float32, seed=19)
    b = _rand((D,), dev, torch.float32, seed=20)
    hi_r, lo_r = _split_ref(res)
    hi = (hi_r.to(torch.int32).to(torch.int16)).view(torch.bfloat16).clone()
    lo = lo_r.to(torch.int32).to(torch.int16).clone()
    assert torch.equal(ops.join_split(hi, lo), res)  # host decode of the host encode
    if mode == "nores":
        ref = F.layer_norm(x.float(), (D,), w, b, 1e-5)
        lib = ops._lib.load()
        hh, ll = torch.empty_like(hi), torch.empty_like(lo)
        ops.check(lib.rf_add_layernorm_split_fwd(M, D, x.data_ptr(), D, None, None, w.data_ptr(), b.data_ptr(),
                                                 1e-5, hh.data_ptr(), ll.data_ptr(), None,
                                                 torch.cuda.current_stream().cuda_stream), "split")
        assert (ops.join_split(hh, ll) - ref).abs().max().item() <= 1e-4
        return
    ref = F.layer_norm(x.float() + res, (D,), w, b, 1e-5)
    yh, yl, y32 = ops.add_layernorm_split(x, hi, lo, w, b, 1e-5, planes=mode != "f32",
                                          want_f32=mode != "planes")
    if mode != "planes":
        assert (y32 - ref).abs().max().item() <= 1e-4
    if mode != "f32":
        assert yh.data_ptr() == hi.data_ptr() and yl.data_ptr() == lo.data_ptr()  # in place
        joined = ops.join_split(yh, yl)
        assert (joined - ref).abs().max().item() <= 1e-4
        if mode == "both":
            assert torch.equal(joined, y32)
        eh, el = _split_ref(joined)
        assert torch.equal(yh.view(torch.int16).long() & 0xFFFF, eh)
        ulp = 2.0 ** (torch.floor(torch.log2(joined.abs().clamp_min(1e-30))) - 7)
        assert ((yh.float() - joined).abs() <= 0.5 * ulp + 1e-30).all()


def test_embed_ln_split(dev):
    from recformer_amd.synth import synth_batch
    B, L, D, V = 2, 128, 768, 500
    bt = {k: v.to(dev) for k, v in synth_batch(B, L, V, seed=5, lens=[128, 77]).items()}
    ids, pos, tt, ip, flags, gidx = ops.prepare_inputs(
        bt["input_ids"], bt["attention_mask"], bt["global_attention_mask"], bt["token_type_ids"],
        bt["item_position_ids"], None, L, 1, 1)
    tabs = [_rand((n, D), dev, torch.float32, 0.02, seed=30 + i) for i, n in enumerate((V, 300, 4, 51))]
    lw = _rand((D,), dev, torch.float32, seed=40)
    lb = _rand((D,), dev, torch.float32, seed=41)
    _, out32 = ops.embed_ln(ids, pos, tt, ip, *tabs, lw, lb, 1e-5, out_dtype=torch.bfloat16, want_f32=True)
    hi, lo = ops.embed_ln_split(ids, pos, tt, ip, *tabs, lw, lb, 1e-5)
    assert torch.equal(ops.join_split(hi, lo), out32)


@pytest.mark.parametrize("tdt,dt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
def test_embed_ln_and_prepare(dev, tdt, dt):
    from recformer_amd.synth import synth_batch
    B, L, D, V = 3, 200, 768, 500
    bt = synth_batch(B, L, V, seed=3, lens=[200, 130, 7], extra_globals=((0, 9), (1, 50)))
    bt = {k: v.to(dev) for k, v in bt.items()}
    Lp = 256
    gmax = 2
    ids, pos, tt, ip, flags, gidx = ops.prepare_inputs(
        bt["input_ids"], bt["attention_mask"], bt["global_attention_mask"], bt["token_type_ids"],
        bt["item_position_ids"], None, Lp, 1, gmax)
    ids_r, merged, tt_r, ip_r, pad = R.prepare_inputs(*(bt[k].cpu() for k in (
        "input_ids", "attention_mask", "global_attention_mask", "token_type_ids", "item_position_ids")), 64, 1)
    assert torch.equal(ids.cpu().long(), ids_r) and torch.equal(tt.cpu().long(), tt_r)
    assert torch.equal(ip.cpu().long(), ip_r)
    ref_flags = torch.where(merged > 1, 2, torch.where(merged == 1, 1, 0))
    assert torch.equal(flags.cpu().long(), ref_flags)
    m = (ids_r != 1).int()
    pos_r = (torch.cumsum(m, 1) * m).long() + 1
    assert torch.equal(pos.cpu().long(), pos_r)
    assert gidx.cpu().tolist() == [[0, 9], [0, 50], [0, -1]]
    tabs = [_rand((n, D), dev, tdt, 0.02, seed=10 + i) for i, n in enumerate((V, 300, 4, 51))]
    lw = _rand((D,), dev, torch.float32, seed=20)
    lb = _rand((D,), dev, torch.float32, seed=21)
    out, out32 = ops.embed_ln(ids, pos, tt, ip, *tabs, lw, lb, 1e-5, out_dtype=dt, want_f32=True)
    x = (tabs[0].float()[ids.long()] + tabs[1].float()[pos.long()] + tabs[2].float()[tt.long()]
         + tabs[3].float()[ip.long()])
    ref = F.layer_norm(x, (D,), lw, lb, 1e-5).view(-1, D)
    tol = 1e-4 if dt == torch.float32 else 2 ** -8 * ref.abs().max().item()
    assert (out.float() - ref).abs().max().item() <= tol
    assert (out32 - ref).abs().max().item() <= 1e-4


def _attn_case(dev, dt, B, Lp, H, lens, globals_, seed):
    D = H * 64
    qkv = _rand((B * Lp, 5 * D), dev, dt, 1.0, seed=seed)
    merged = torch.zeros(B, Lp, dtype=torch.long)
    for b, n in enumerate(lens):
        merged[b, :n] = 1
    for b, p in globals_:
        if p < lens[b]:
            merged[b, p] = 2
    flags = merged.to(torch.uint8).to(dev)
    G = int((merged > 1).sum(1).max())
    gidx = torch.full((B, max(G, 1)), -1, dtype=torch.int32)
    for b in range(B):
        pos = torch.nonzero(merged[b] > 1).flatten()
        gidx[b, :pos.numel()] = pos.int()
    gidx = gidx[:, :G].to(dev)
    return qkv, merged, flags, gidx, G


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=2, Lp=256, H=2, lens=[256, 100], globals_=((0, 0), (1, 0))),
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=1, Lp=128, H=1, lens=[128], globals_=()),
    dict(B=1, Lp=1024, H=12, lens=[1024], globals_=((0, 0),)),
])
def test_band_and_global_attention(dev, dt, case):
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 7)
    q, k, v, kg, vg = (qkv[:, i * D:(i + 1) * D] for i in range(5))
    ctx = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32)
    qg = None
    if G:
        qg_rows = _rand((B * G, D), dev, dt, 1.0, seed=8)
        ops.global_attention(qg_rows, kg, vg, flags, gidx, B, Lp, H, ctx)
        qg = qg_rows.float().cpu().view(B, G, H, 64).transpose(1, 2)

    def hv(x):
        return x.float().cpu().view(B, Lp, H, 64).transpose(1, 2)

    ref = R.band_global_attention(hv(q), hv(k), hv(v), merged, 32, qg,
                                  hv(kg) if G else None, hv(vg) if G else None)
    ref = ref.transpose(1, 2).reshape(B * Lp, D)
    err = (ctx.float().cpu() - ref).abs().max().item()
    assert err <= (1e-4 if dt == torch.float32 else 3e-2), err
    # padded query rows are exactly zero
    pad_rows = (merged.view(-1) == 0)
    assert ctx.float().cpu()[pad_rows].abs().max().item() == 0.0 if pad_rows.any() else True


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(half_w=256, B=2, Lp=1024, H=2, lens=[1024, 700], globals_=((0, 0), (1, 0), (1, 500))),
    dict(half_w=64, B=2, Lp=384, H=3, lens=[384, 200], globals_=((0, 0),)),
    dict(half_w=20, B=2, Lp=200, H=2, lens=[200, 57], globals_=((0, 0), (1, 3))),
    dict(half_w=96, B=1, Lp=576, H=1, lens=[576], globals_=tuple((0, 13 * i) for i in range(40))),
])
def test_band_attention_other_windows(dev, dt, case):
    """16-bit local attention at windows other than 64 (k_band_attn_wide: the reference accepts any
    even per-layer window, models.py:179-187) against the oracle, incl. Lp not a multiple of 64 and
    more than 32 global keys; then the global rows through rf_global_attn_fwd."""
    B, Lp, H, hw = case["B"], case["Lp"], case["H"], case["half_w"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 17)
    q, k, v, kg, vg = (qkv[:, i * D:(i + 1) * D] for i in range(5))
    ctx = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, hw)
    qg = None
    if G:
        qg_rows = _rand((B * G, D), dev, dt, 1.0, seed=18)
        ops.global_attention(qg_rows, kg, vg, flags, gidx, B, Lp, H, ctx)
        qg = qg_rows.float().cpu().view(B, G, H, 64).transpose(1, 2)

    def hv(x):
        return x.float().cpu().view(B, Lp, H, 64).transpose(1, 2)

    ref = R.band_global_attention(hv(q), hv(k), hv(v), merged, hw, qg,
                                  hv(kg) if G else None, hv(vg) if G else None)
    ref = ref.transpose(1, 2).reshape(B * Lp, D)
    err = (ctx.float().cpu() - ref).abs().max().item()
    assert err <= 3e-2, err
    pad_rows = merged.view(-1) == 0
    if pad_rows.any():
        assert ctx.float().cpu()[pad_rows].abs().max().item() == 0.0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_cos_scores(dev, dt):
    z = _rand((37, 768), dev, dt, seed=30)
    E = _rand((1000, 768), dev, dt, seed=31)
    s = ops.cos_scores(z, E, 20.0)
    ref = F.cosine_similarity(z.float().unsqueeze(1), E.float().unsqueeze(0), dim=-1) * 20.0
    assert (s - ref).abs().max().item() <= (1e-4 if dt == torch.float32 else 2e-2)
    cand = torch.randint(0, 1000, (37, 65), device=dev)
    sc = ops.cos_scores_cand(z, E, cand, 20.0)
    refc = torch.gather(ref, 1, cand)
    assert (sc - refc).abs().max().item() <= (1e-4 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=2, Lp=256, H=2, lens=[256, 100], globals_=((0, 0), (1, 0))),
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=2, Lp=1024, H=12, lens=[1024, 333], globals_=((0, 0), (1, 0))),
])
def test_global_attention_fold(dev, dt, case):
    """Fold form (u = Wkg^T qg over h, out = Wvg (sum p h) + b) vs the reference structure
    (k_g = Wkg h + b over all tokens, softmax, p . v_g), both on the same inputs in fp32."""
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    _, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=40)
    wkg = _rand((D, D), dev, dt, 0.05, seed=41)
    wvg = _rand((D, D), dev, dt, 0.05, seed=42)
    bkg = _rand((D,), dev, torch.float32, 0.1, seed=43)
    bvg = _rand((D,), dev, torch.float32, 0.1, seed=44)
    qg = _rand((B * G, D), dev, dt, 1.0, seed=45)
    ctx = torch.zeros(B * Lp, D, dtype=dt, device=dev)
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx)
    hf = h.float().cpu()
    kg = (hf @ wkg.float().cpu().t() + bkg.cpu()).view(B, Lp, H, 64).transpose(1, 2)
    vg = (hf @ wvg.float().cpu().t() + bvg.cpu()).view(B, Lp, H, 64).transpose(1, 2)
    q = qg.float().cpu().view(B, G, H, 64).transpose(1, 2)
    valid = (merged > 0)
    s = torch.matmul(q, kg.transpose(-1, -2)).masked_fill(~valid.view(B, 1, 1, Lp), float("-inf"))
    og = torch.matmul(torch.softmax(s, -1), vg)                 # (B,H,G,64)
    got = ctx.float().cpu().view(B, Lp, H, 64)
    gl = gidx.cpu()
    for b in range(B):
        for g in range(G):
            p = int(gl[b, g])
            if p < 0:
                continue
            err = (got[b, p] - og[b, :, g]).abs().max().item()
            assert err <= (1e-4 if dt == torch.float32 else 2e-2), (b, g, err)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N", [4, 1000, 50265])
def test_cross_entropy(dev, dt, N):
    """rf_cross_entropy_fwd vs torch cross_entropy (mean over non-ignored, ignore -100) + argmax."""
    torch.manual_seed(N)
    M = 37
    x = (torch.randn(M, N, device=dev) * 3).to(dt)
    lab = torch.randint(0, N, (M,), device=dev)
    lab[::5] = -100
    loss, am = ops.cross_entropy(x, lab, want_argmax=True)
    ref = F.cross_entropy(x.float(), lab, ignore_index=-100)
    assert abs(float(loss) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    assert torch.equal(am, x.float().argmax(1))
    rows = ops.cross_entropy(x, lab, reduction="none")
    refr = F.cross_entropy(x.float(), lab, ignore_index=-100, reduction="none")
    assert (rows - refr).abs().max().item() <= 1e-4
    # strided (padded leading dim) logits view
    xp = torch.zeros(M, N + 5, device=dev, dtype=dt)
    xp[:, :N] = x
    assert abs(float(ops.cross_entropy(xp[:, :N], lab)) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=2, Lp=1024, H=12, lens=[1024, 333], globals_=((0, 0), (1, 0))),
])
def test_global_attention_fold_from_h(dev, dt, case):
    """rf_global_attn_fold_h_fwd (query_global projection of the gathered rows + fold in one
    entry point) against gather + qg GEMM + rf_global_attn_fold_fwd on the same inputs."""
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    _, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=50)
    wqg = _rand((D, D), dev, dt, 0.05, seed=51)
    wkg = _rand((D, D), dev, dt, 0.05, seed=52)
    wvg = _rand((D, D), dev, dt, 0.05, seed=53)
    bqg = _rand((D,), dev, torch.float32, 0.1, seed=54)
    bkg = _rand((D,), dev, torch.float32, 0.1, seed=55)
    bvg = _rand((D,), dev, torch.float32, 0.1, seed=56)
    scale = 0.125
    ctx_a = torch.zeros(B * Lp, D, dtype=dt, device=dev)
    ops.global_attention_fold_h(h, wqg, bqg, scale, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx_a)
    hg = ops.gather_global_rows(h, gidx, B, Lp)
    qg = ops.gemm(hg, wqg, bqg, ops.RF_EPI_BIAS, scale_cols=D, col_scale=scale)
    ctx_b = torch.zeros(B * Lp, D, dtype=dt, device=dev)
    ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, ctx_b)
    err = (ctx_a.float() - ctx_b.float()).abs().max().item()
    assert err <= (1e-4 if dt == torch.float32 else 2e-2), err
    assert ctx_a.abs().sum().item() > 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Lp,H", [(3, 192, 3), (4, 1024, 12), (300, 64, 12)])
def test_global_fold_h_stages_match_one_call(dev, dt, B, Lp, H):
    """rf_global_attn_fold_h_stage(1) then (2) — as the encoder runs it, with h overwritten in
    between (stage 2 must read only the workspace) and out untouched by stage 1 — is bit-identical
    to the one-call rf_global_attn_fold_h_fwd."""
    D = H * 64
    g = torch.Generator().manual_seed(B + Lp)
    lens = [int(x) for x in torch.randint(1, Lp + 1, (B,), generator=g)]
    lens[0] = Lp
    globals_ = [(b, 0) for b in range(B) if b % 5 != 2] + [(b, lens[b] - 1) for b in range(0, B, 3)]
    _, _, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, lens, globals_, 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=70)
    w = [_rand((D, D), dev, dt, 0.05, seed=71 + i) for i in range(3)]
    bias = [_rand((D,), dev, torch.float32, 0.1, seed=74 + i) for i in range(3)]
    args = (w[0], bias[0], 0.125, w[1], bias[1], w[2], bias[2], flags, gidx, B, Lp, H)
    ref = torch.full((B * Lp, D), 3.0, dtype=dt, device=dev)
    ops.global_attention_fold_h(h, *args, ref)
    ws = ops.global_fold_workspace(h, B, Lp, H, gidx.shape[1])
    out = torch.full((B * Lp, D), 3.0, dtype=dt, device=dev)
    ops.global_attention_fold_h_stage(1, ws, h, *args)
    h_keep = h.clone()
    h.normal_()
    ops.global_attention_fold_h_stage(2, ws, h, *args, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    with pytest.raises(ValueError):
        ops.global_attention_fold_h_stage(2, ws, h_keep, *args)


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Lp,H", [(3, 192, 3), (4, 1024, 12)])
def test_global_fold_fwd_stages_match_fused(dev, dt, B, Lp, H, p_drop):
    """rf_global_attn_fold_fwd_stage(1) then (2) on one workspace — how the training forward runs the
    fold beside the band attention (train.FOLD_SIDE_TRAIN) — is bit-identical to the one-call stage 3,
    with and without attention dropout; stage 1 leaves out untouched and stage 2 reads only the
    workspace (h overwritten in between)."""
    D = H * 64
    g = torch.Generator().manual_seed(B * Lp + H)
    lens = [int(x) for x in torch.randint(1, Lp + 1, (B,), generator=g)]
    lens[0] = Lp
    globals_ = [(b, 0) for b in range(B)] + [(b, lens[b] - 1) for b in range(0, B, 2)]
    _, _, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, lens, globals_, 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=80)
    wkg = _rand((D, D), dev, dt, 0.05, seed=81)
    wvg = _rand((D, D), dev, dt, 0.05, seed=82)
    bkg = _rand((D,), dev, torch.float32, 0.1, seed=83)
    bvg = _rand((D,), dev, torch.float32, 0.1, seed=84)
    qg = _rand((B * G, D), dev, dt, 1.0, seed=85)
    args = (wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H)
    ref = torch.full((B * Lp, D), 3.0, dtype=dt, device=dev)
    ws3 = ops.global_fold_workspace(h, B, Lp, H, gidx.shape[1])
    ops.global_attention_fold(qg, h, *args, ref, p_drop=p_drop, seed=1234, ws=ws3, stage=3)
    ws = ops.global_fold_workspace(h, B, Lp, H, gidx.shape[1])
    out = torch.full((B * Lp, D), 3.0, dtype=dt, device=dev)
    ops.global_attention_fold(qg, h, *args, None, p_drop=p_drop, seed=1234, ws=ws, stage=1)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.full_like(out, 3.0))
    h.normal_()
    ops.global_attention_fold(qg, h, *args, out, p_drop=p_drop, seed=1234, ws=ws, stage=2)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert (out != 3.0).any()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Lp,H", [(300, 64, 12), (70, 192, 3), (5, 1024, 12)])
def test_global_fold_mfma_matches_gemv(dev, monkeypatch, B, Lp, H, dt):
    """The 64-row MFMA qg/u and out kernels (chosen for >= 256 global rows, e.g. a catalog of
    short item sequences), the default choice (below 256 rows: the 16-row MFMA out kernel
    k_gfold_out16) and the two-half partial kernel the 32-row ring replaced (knob 3) against the
    per-row GEMV kernels (pinned to the torch reference by
    test_band_and_global_attention) on the same inputs: ragged lengths, sequences without a
    global token (gidx -1), several globals per sequence and partial last 64- / 16-row tiles."""
    D = H * 64
    g = torch.Generator().manual_seed(B)
    lens = [int(x) for x in torch.randint(1, Lp + 1, (B,), generator=g)]
    lens[0] = Lp
    globals_ = [(b, 0) for b in range(B) if b % 7 != 3] + [(b, lens[b] - 1) for b in range(0, B, 5)]
    _, _, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, lens, globals_, 3)
    h = _rand((B * Lp, D), dev, dt, 1.0, seed=60)
    w = [_rand((D, D), dev, dt, 0.05, seed=61 + i) for i in range(3)]
    bias = [_rand((D,), dev, torch.float32, 0.1, seed=64 + i) for i in range(3)]
    outs = {}
    for path in ("gemv", "mfma", "auto", "two_half"):
        old = _lib.set_knob("gfold_path", {"gemv": 1, "mfma": 2, "auto": 0, "two_half": 3}[path])
        ctx = torch.zeros(B * Lp, D, dtype=dt, device=dev)
        ops.global_attention_fold_h(h, w[0], bias[0], 0.125, w[1], bias[1], w[2], bias[2], flags, gidx, B, Lp, H,
                                    ctx)
        torch.cuda.synchronize()
        _lib.set_knob("gfold_path", old)
        outs[path] = ctx.float()
    for other in ("mfma", "auto", "two_half"):
        err = (outs["gemv"] - outs[other]).abs().max().item()
        assert err <= 2e-2, (other, err)
    written = outs["auto"].abs().sum(1) > 0
    assert int(written.sum()) == int((gidx >= 0).sum())  # exactly the global rows are overwritten


@pytest.mark.parametrize("N", [7, 1000, 100003])
def test_ranker_matches_reference_formula(dev, N):
    """Ranker (rf_rank_accum + rf_cross_entropy_fwd) vs utils.py:76-108 restated (oracle), with
    ties, masked (-MAX_VAL) columns and labels at the extremes."""
    from recformer_amd import Ranker
    torch.manual_seed(N)
    B = 33
    s = torch.randn(B, N) * 4
    s[:, ::7] = torch.round(s[:, ::7])  # ties
    s[3, : N // 2] = -2e4                # masked part of a row (valid_length < N)
    labels = torch.randint(0, N, (B,))
    labels[0], labels[1] = 0, N - 1
    s[5, labels[5]] = s[5].max()        # rank 0
    ref = R.ranker_metrics(s.clone(), labels.clone(), [1, 10, 50])
    got = Ranker([1, 10, 50])(s.to(dev), labels.to(dev))
    assert len(got) == len(ref)
    for g, r in zip(got[:-1], ref[:-1]):
        assert abs(g - r) <= 1e-6, (got, ref)
    assert abs(got[-1] - ref[-1]) <= 1e-5 * max(1.0, abs(ref[-1]))


@pytest.mark.parametrize("case", ["ties", "masked", "cosine"])
def test_ranker_matches_reference_fixture(dev, case):
    """Ranker on the device vs the real Ranker's outputs (tests/golden/ranker.npz made by
    oracle/gen_golden_ranker.py from utils.py:76-108): exact ranks, ties, -MAX_VAL, B = 37."""
    from recformer_amd import Ranker
    from recformer_amd.ranker import rank_counts
    from tests.common import load_golden
    g = load_golden("ranker")
    ks = [int(k) for k in g["ks"]]
    s, lab = g[f"{case}_scores"], g[f"{case}_labels"]
    gt, valid = rank_counts(s.to(dev), lab.to(dev))
    assert torch.equal(gt.cpu().long(), g[f"{case}_rank"].long())
    assert torch.equal(valid.cpu().long(), g[f"{case}_valid"].long())
    got = Ranker(ks)(s.to(dev), lab.to(dev))
    ref = g[f"{case}_metrics"].tolist()
    for a, b in zip(got[:-1], ref[:-1]):
        assert a == pytest.approx(b, abs=1e-6)
    assert got[-1] == pytest.approx(ref[-1], rel=1e-5)


@pytest.mark.parametrize("B,N,block,dts", [(37, 1000, 1000, "bf16"), (37, 5003, 2048, "bf16"),
                                          (37, 5003, 2048, "fp32"), (37, 1000, 1000, "fp32"),
                                          (37, 5003, 2048, "mixed")])
def test_rank_catalog_matches_restated_ranker(dev, B, N, block, dts):
    """rank_catalog against utils.py:76-108 restated (oracle, pinned by tests/golden/ranker.npz)
    on the same fp32 cosine-score matrix: B not a multiple of 16, ragged column tails, every third
    label in the last partial 16 columns of the catalog (or of a block), exact duplicate items.
    fp32 (an fp32 model's pooler output and catalog) and mixed-dtype inputs take the exact-fp32
    block path; its scores are the EPI_COS fp32 GEMM's, the same the reference matrix is made of."""
    from recformer_amd.ranker import rank_catalog
    g = torch.Generator(device=dev).manual_seed(B * N)
    qdt = torch.bfloat16 if dts == "bf16" else torch.float32
    idt = torch.float32 if dts == "fp32" else torch.bfloat16
    q = torch.randn(B, 768, device=dev, generator=g).to(qdt)
    items = torch.randn(N, 768, device=dev, generator=g).to(idt)
    labels = torch.randint(0, N, (B,), device=dev, generator=g)
    labels[::3] = N - 1 - torch.arange(len(labels[::3]), device=dev) % 8
    labels[1::3] = (block - 1 - torch.arange(len(labels[1::3]), device=dev) % 8) % N
    dup = labels[:8]
    items[(dup + N // 2) % N] = items[dup]
    if q.dtype != items.dtype:
        s = ops.cos_scores(q.float(), items.float(), 20.0).cpu()
    else:
        s = ops.cos_scores(q, items, 20.0).cpu()
    ref = R.ranker_metrics(s, labels.cpu(), [1, 10, 50])
    got = rank_catalog(q, items, labels, [1, 10, 50], 0.05, block=block)
    for a, b in zip(got[:-1], ref[:-1]):
        assert a == pytest.approx(b, abs=1e-6), (got, ref)
    assert got[-1] == pytest.approx(ref[-1], rel=1e-4)


def test_retrieval_topk_argument_checks(dev):
    """k / sample outside the top-k kernels' limits fail with a clear ValueError (not a kernel error)."""
    from recformer_amd.ranker import CatalogShard, retrieve, shard_rank
    items = torch.randn(300, 64, device=dev).to(torch.float16)
    q = torch.randn(4, 64, device=dev).to(torch.float16)
    shard = CatalogShard(items)
    sl = torch.zeros(4, device=dev)
    for kw in (dict(k=257), dict(k=50, sample=4096), dict(k=50, sample=10)):
        with pytest.raises(ValueError):
            shard_rank(q, shard, sl, 0.05, **kw)
    with pytest.raises(ValueError):
        retrieve(q, shard, torch.zeros(4, dtype=torch.int64, device=dev), [10], 0.05, k=300)


@pytest.mark.parametrize("M,D", [(333, 768), (64, 128), (1000, 1024)])
def test_layernorm_bwd_matches_autograd(dev, M, D):
    """rf_layernorm_bwd vs torch autograd of F.layer_norm in fp32 (training path, TF:1071)."""
    x = _rand((M, D), dev, torch.float32, 2.0, seed=31) + 0.3
    w = _rand((D,), dev, torch.float32, seed=32)
    b = _rand((D,), dev, torch.float32, seed=33)
    dy = _rand((M, D), dev, torch.float32, seed=34)
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.layer_norm(xr, (D,), wr, br, 1e-5).backward(dy)
    _, mean, rstd = ops.layernorm(x, w, b, 1e-5, stats=True)
    dx, dw, db = ops.layernorm_bwd(dy, x, mean, rstd, w)
    assert (dx - xr.grad).abs().max().item() <= 1e-4 * xr.grad.abs().max().item() + 1e-5
    assert (dw - wr.grad).abs().max().item() <= 1e-4 * wr.grad.abs().max().item() + 1e-4
    assert (db - br.grad).abs().max().item() <= 1e-4 * br.grad.abs().max().item() + 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N", [(1, 5), (333, 768), (16384, 2304), (70, 3072), (65, 6)])
def test_colsum(dev, dt, M, N):
    for x in (_rand((M, N + 8), dev, dt, seed=41)[:, :N], _rand((M, N + 3), dev, dt, seed=42)[:, :N]):
        ref = x.float().sum(0)  # strided rows: vector path (ld % 4 == 0) and scalar path
        out = ops.colsum(x)
        assert (out - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item()) + 1e-3
        # the first columns under a power-of-two scale (the query's 1/8): exactly the scaled sums
        sc = (N + 1) // 2
        exp = out.clone()
        exp[:sc] *= 0.125
        assert torch.equal(ops.colsum(x, sc, 0.125), exp)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_drop_add_ln_matches_torch(dev, p):
    """Fused dropout + residual + LayerNorm (training path): with the keep mask recovered from the
    saved pre-LN rows, forward and every gradient match torch autograd of the same composition;
    the keep fraction is 1 - p."""
    M, D = 512, 768
    t = _rand((M, D), dev, torch.bfloat16, 1.0, seed=51)
    res = _rand((M, D), dev, torch.float32, 1.0, seed=52)
    w = _rand((D,), dev, torch.float32, seed=53)
    b = _rand((D,), dev, torch.float32, seed=54)
    dy = _rand((M, D), dev, torch.float32, seed=55)
    x, y, mean, rstd = ops.drop_add_ln_fwd(t, res, w, b, 1e-5, p, 12345)
    scaled = t.float() / (1 - p)
    keep = ((x - res) - scaled).abs() <= 1e-5 * scaled.abs() + 1e-6
    zero = (x - res).abs() <= 1e-6
    assert bool((keep | zero).all())
    if p > 0:
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.01, frac
    else:
        assert bool(keep.all())
    mask = keep.float()
    tr, rr = t.float().clone().requires_grad_(True), res.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(tr * mask / (1 - p) + rr, (D,), wr, br, 1e-5)
    yr.backward(dy)
    assert (y - yr).abs().max().item() <= 1e-4
    dres, dt, dw, db = ops.drop_add_ln_bwd(dy, x, mean, rstd, w, p, 12345)
    assert (dres - rr.grad).abs().max().item() <= 1e-4 * rr.grad.abs().max().item() + 1e-5
    assert (dt.float() - tr.grad).abs().max().item() <= 2 ** -7 * tr.grad.abs().max().item()
    assert (dw - wr.grad).abs().max().item() <= 1e-4 * wr.grad.abs().max().item() + 1e-4
    assert (db - br.grad).abs().max().item() <= 1e-4 * br.grad.abs().max().item() + 1e-4


@pytest.mark.parametrize("D", [768, 256])
def test_drop_add_ln_dual(dev, D):
    """rf_drop_add_ln_fwd_dual / _bwd_dual (the training path's LayerNorm feeding both the next
    residual add and the next GEMM): y16 is bf16(y) bit for bit, and the backward with the two
    consumers' gradients (fp32 dy, bf16 dy16; either alone) equals the single-gradient backward
    of dy + float(dy16)."""
    M = 300
    g = torch.Generator(device=dev).manual_seed(D)
    t = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    res = torch.randn(M, D, device=dev, generator=g)
    w = torch.rand(D, device=dev, generator=g) + 0.5
    b = torch.randn(D, device=dev, generator=g) * 0.1
    x, y, mean, rstd, y16 = ops.drop_add_ln_fwd(t, res, w, b, 1e-5, 0.1, 1234, want_bf16=True)
    x1, y1, _, _ = ops.drop_add_ln_fwd(t, res, w, b, 1e-5, 0.1, 1234)
    assert torch.equal(y16, y.to(torch.bfloat16)) and torch.equal(y, y1) and torch.equal(x, x1)
    dy = torch.randn(M, D, device=dev, generator=g)
    dy16 = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    cases = ((dy, dy16, dy + dy16.float()), (None, dy16, dy16.float()), (dy, None, dy))
    for a, c, ref_dy in cases:
        got = ops.drop_add_ln_bwd(a, x, mean, rstd, w, 0.1, 1234, dy16=c)
        ref = ops.drop_add_ln_bwd(ref_dy, x, mean, rstd, w, 0.1, 1234)
        for u, v in zip(got, ref):
            assert torch.equal(u, v)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float16])
def test_scatter_add_rows(dev, dt):
    """rf_scatter_add_rows: dst[rows[r]] += src[r] for two pairs, strided destinations (column
    views of one wide tensor), skipped rows (-1) and a repeated row, against index_add_."""
    g = torch.Generator(device=dev).manual_seed(5)
    R, D, M = 9, 768, 50
    rows = torch.tensor([3, -1, 7, 3, 0, 49, -1, 12, 7], dtype=torch.int32, device=dev)
    src = [torch.randn(R, D, device=dev, generator=g).to(dt) for _ in range(2)]
    wide = torch.randn(M, 3 * D, device=dev, generator=g).to(dt)
    ref = wide.clone()
    keep = rows >= 0
    for i, s in enumerate(src):
        col = ref[:, (i + 1) * D:(i + 2) * D].float()
        col.index_add_(0, rows[keep].long(), s[keep].float())
        ref[:, (i + 1) * D:(i + 2) * D] = col.to(dt)
    ops.scatter_add_rows(rows, src[0], wide[:, D:2 * D], src[1], wide[:, 2 * D:])
    torch.cuda.synchronize()
    tol = 1e-5 if dt == torch.float32 else 1e-2  # repeated rows: addition order may differ
    assert float((wide.float() - ref.float()).abs().max()) <= tol * 8
    assert torch.equal(wide[:, :D], ref[:, :D])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (8192, 768, 3072), (4100, 2304, 768)])
@pytest.mark.parametrize("epi", [ops.RF_EPI_NONE, ops.RF_EPI_BIAS, ops.RF_EPI_BIAS_GELU, ops.RF_EPI_BIAS_RESID,
                                 ops.RF_EPI_COS])
def test_gemm_pingpong_16bit(dev, dt, M, N, K, epi):
    """The 256x256 ping-pong kernel (grids >= 128 tiles) in bf16 and fp16 for every epilogue,
    including a ragged M edge, against fp32 torch on the same operands."""
    a = _rand((M, K), dev, dt, 0.5, seed=81)
    w = _rand((N, K), dev, dt, 0.05, seed=82)
    b = _rand((N,), dev, torch.float32, seed=83)
    r = _rand((M, N), dev, dt, seed=84)
    if epi == ops.RF_EPI_COS:
        ra = (1.0 / a.float().norm(dim=-1).clamp_min(1e-8)).contiguous()
        rw = (1.0 / w.float().norm(dim=-1).clamp_min(1e-8)).contiguous()
        out = ops.cos_scores(a, w, 20.0, z_rnorm=ra, items_rnorm=rw)
        ref = F.normalize(a.float(), dim=-1) @ F.normalize(w.float(), dim=-1).t() * 20.0
        assert (out - ref).abs().max().item() <= 2e-2
        return
    out = ops.gemm(a, w, b if epi else None, epi, resid=r if epi == ops.RF_EPI_BIAS_RESID else None,
                   scale_cols=N // 3 // 16 * 16, col_scale=0.125)
    ref = a.float() @ w.float().t()
    if epi:
        ref = ref + b
    ref[:, :N // 3 // 16 * 16] *= 0.125
    if epi == ops.RF_EPI_BIAS_GELU:
        ref = F.gelu(ref)
    if epi == ops.RF_EPI_BIAS_RESID:
        ref = ref + r.float()
    rel = (out.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert rel <= (4e-3 if dt == torch.float16 else 2e-2), rel


@pytest.mark.parametrize("M,N", [(4096, 3072), (1000, 3072), (300, 200)])
def test_gemm_gelu_aux(dev, M, N):
    """EPI_BIAS_GELU_AUX (training FFN1): C equals the EPI_BIAS_GELU output and the written
    pre-activation equals the EPI_BIAS output, bit for bit, on the ping-pong (large), tiled
    (small) and ragged-edge paths."""
    K = 768
    g = torch.Generator(device=dev).manual_seed(M + N)
    a = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g) * 0.1
    z = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    u = ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
    assert torch.equal(u, ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU))
    assert torch.equal(z, ops.gemm(a, w, b, ops.RF_EPI_BIAS))


@pytest.mark.parametrize("B,N,block", [(256, 20000, 8192), (4096, 66536, 65536), (64, 1000, 1000)])
def test_rank_catalog_matches_full_ranker(dev, B, N, block):
    """ranker.rank_catalog (scores block by block, never the (B, N) matrix) gives the full-matrix
    Ranker's metrics: identical strict ranks (the label scores are the same kernel's values), the
    loss within fp32 rounding of the two log-sum-exp forms."""
    from recformer_amd import Ranker
    from recformer_amd.ranker import rank_catalog
    g = torch.Generator(device=dev).manual_seed(B + N)
    q = torch.randn(B, 768, device=dev, generator=g).to(torch.bfloat16)
    items = torch.randn(N, 768, device=dev, generator=g).to(torch.bfloat16)
    labels = torch.randint(0, N, (B,), device=dev, generator=g)
    # exact ties: copies of some label items elsewhere in the catalog (strict ranks ignore them)
    dup = labels[: min(B, 16)]
    items[(dup + N // 2) % N] = items[dup]
    full = Ranker([10, 50])(ops.cos_scores(q, items, 20.0), labels)
    got = rank_catalog(q, items, labels, [10, 50], 0.05, block=block)
    assert got[:-1] == full[:-1]
    assert got[-1] == pytest.approx(full[-1], rel=1e-5, abs=1e-5)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (1000, 384, 192), (300, 256, 64)])
def test_gemm_dgelu_epilogue(dev, dt, M, N, K):
    """EPI_DGELU: C = (A.W^T) * gelu'(R) (the GELU backward fused into the next Linear's dA GEMM)
    against torch's gelu_backward of the fp32 product on the same operands."""
    a = _rand((M, K), dev, dt, 1.0, seed=61)
    w = _rand((N, K), dev, dt, 0.1, seed=62)
    z = _rand((M, N), dev, dt, 2.0, seed=63)
    out = ops.gemm(a, w, None, ops.RF_EPI_DGELU, resid=z)
    ref = torch.ops.aten.gelu_backward(a.float() @ w.float().t(), z.float())
    err = float((out.float() - ref).abs().max())
    assert err <= 1e-2 * max(float(ref.abs().max()), 1e-6), err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K,strided", [(16384, 2304, 768, False), (16384, 768, 3072, False),
                                           (16384, 3072, 768, False), (1000, 768, 768, True), (333, 64, 128, False),
                                           (70000, 768, 768, False), (64, 256, 272, False), (4, 768, 768, False),
                                           (16, 3072, 768, False), (1, 64, 128, False)])
def test_weight_grad_matches_fp32_matmul(dev, dt, M, N, K, strided):
    """rf_weight_grad (dW = dC^T A on MFMA with transposed LDS reads, rows split over workgroups and
    reduced in a fixed order) against torch's fp32 product of the same 16-bit operands: products of
    16-bit values are exact in fp32, only the summation order differs (<= 1e-4 x max|dW|); ragged M
    (not a multiple of 64 or of the split), N / K not multiples of 256, a strided column-slice dC (the
    fused q|k|v gradient's layout); bit-identical on a repeat (deterministic); accumulate adds."""
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    if strided:
        big = torch.randn(M, 3 * N, device=dev, generator=g).to(dt)
        dc = big[:, N:2 * N]
    else:
        dc = torch.randn(M, N, device=dev, generator=g).to(dt)
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    ref = dc.float().t() @ a.float()
    got = ops.weight_grad(dc, a)
    err = float((got - ref).abs().max())
    assert err <= 1e-4 * float(ref.abs().max()) + 1e-5, err
    assert torch.equal(got, ops.weight_grad(dc, a))
    base = torch.randn(N, K, device=dev, generator=g)
    acc = base.clone()
    ops.weight_grad(dc, a, out=acc, accumulate=True)
    assert float((acc - (base + ref)).abs().max()) <= 1e-4 * float(ref.abs().max()) + 1e-5
    # the first rows under a power-of-two scale (the query's 1/8, TF:504-514): exactly the scaled rows
    sr = min(N, 16 * ((N // 3 + 15) // 16))
    exp = got.clone()
    exp[:sr] *= 0.125
    assert torch.equal(ops.weight_grad(dc, a, scale_rows=sr, row_scale=0.125), exp)
    acc2 = base.clone()
    ops.weight_grad(dc, a, out=acc2, accumulate=True, scale_rows=sr, row_scale=0.125)
    assert torch.equal(acc2, base + exp)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [
    dict(B=2, Lp=256, H=2, lens=[256, 100], globals_=((0, 0), (1, 0))),
    dict(B=3, Lp=192, H=3, lens=[192, 150, 1], globals_=((0, 0), (0, 70), (0, 191), (1, 0), (1, 33), (1, 149), (2, 0))),
    dict(B=1, Lp=128, H=1, lens=[128], globals_=()),
    dict(B=2, Lp=1024, H=12, lens=[1024, 700], globals_=((0, 0), (1, 0), (1, 5))),
    dict(B=1, Lp=640, H=2, lens=[600], globals_=tuple((0, 19 * i) for i in range(32))),
])
def test_band_pipe3_bit_identical_to_pipe2(dev, dt, case):
    """The three-workgroups-per-CU band kernel (k_band_attn_pipe3: Q fragments and the global keys'
    K / V^T fragments loaded straight into registers, 48 KB of LDS) computes exactly what
    k_band_attn_pipe2 (pinned to the reference through test_band_and_global_attention) computes:
    same MFMA chain, same softmax, same stores — outputs bit-identical, incl. ragged rows, padded
    rows, up to 32 global keys, one run of 10 query blocks (Lp = 640) and two runs of 8 (Lp = 1024)."""
    from recformer_amd import _lib
    B, Lp, H = case["B"], case["Lp"], case["H"]
    D = H * 64
    qkv, merged, flags, gidx, G = _attn_case(dev, dt, B, Lp, H, case["lens"], case["globals_"], 11)
    q, k, v = (qkv[:, i * D:(i + 1) * D] for i in range(3))
    old = _lib.set_knob("band_path", 0)
    try:
        ref = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32)
        _lib.set_knob("band_path", 3)
        got = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, 32)
    finally:
        _lib.set_knob("band_path", old)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("M,D,V,kind", [
    (1, 768, 50, "uniform"), (33, 768, 50, "uniform"), (5000, 768, 50265, "tokens"), (5000, 100, 300, "tokens"),
    (4096, 1024, 1026, "positions"), (70000, 768, 4, "types"), (70000, 256, 51, "itempos"), (2100, 512, 3, "pad_only"),
])
def test_embedding_grad_matches_index_add(dev, M, D, V, kind):
    """rf_segment_rows_sum (nn.Embedding's dense backward, models.py:82-138) against an fp64 index_add:
    word-like ids with a frequent padding id (1, no gradient at that row) and repeated common tokens,
    position ids, a 4-value type table whose segment spans more than 64 x 256 sorted positions (several
    ballot rounds of 1024-boundary chains), item positions, ragged D (100: not a multiple of 256),
    a single row, and an all-padding input; deterministic (bit-identical on a repeat)."""
    g = torch.Generator(device="cpu").manual_seed(M + D + V)
    if kind == "tokens":
        idx = torch.randint(0, V, (M,), generator=g)
        idx[torch.rand(M, generator=g) < 0.3] = 1
        idx[torch.rand(M, generator=g) < 0.1] = 2
    elif kind == "positions":
        idx = (torch.arange(M) % 1024) + 2
    elif kind == "types":
        idx = torch.zeros(M, dtype=torch.long)
        idx[torch.rand(M, generator=g) < 0.02] = 3
    elif kind == "pad_only":
        idx = torch.ones(M, dtype=torch.long)
    else:
        idx = torch.randint(0, V, (M,), generator=g)
    src = torch.randn(M, D, generator=g)
    pad = None if kind in ("types", "itempos", "uniform") else 1
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, idx, src.double())
    if pad is not None:
        ref[pad] = 0
    got = ops.embedding_grad(src.to(dev), idx.to(dev), V, pad)
    scale = float(ref.abs().max()) if ref.abs().max() > 0 else 1.0
    err = float((got.double().cpu() - ref).abs().max())
    assert err <= 2e-6 * scale * max(1.0, math.log2(M)) + 1e-6, (err, scale)
    assert torch.equal(got, ops.embedding_grad(src.to(dev), idx.to(dev), V, pad))


@pytest.mark.parametrize("M,D", [(1, 768), (3000, 768), (20000, 768), (777, 256), (500, 1024), (300, 100)])
def test_embed_ln_bwd_matches_autograd(dev, M, D):
    """rf_embed_ln_bwd (LayerNorm backward over the regathered 4-table sum, models.py:108-138) against
    fp64 autograd of the same forward: dx and dgamma / dbeta (fixed-order block sums, bit-identical on
    a repeat); then the full _EmbedLN backward (HIP kernels) against its torch path (index_add_)."""
    from recformer_amd import train as T
    g = torch.Generator(device="cpu").manual_seed(M + D)
    Vw, P, Tt, I = 1000, 1026, 4, 51
    word, pe, te, ie = (torch.randn(n, D, generator=g) * 0.5 for n in (Vw, P, Tt, I))
    ids = torch.randint(0, Vw, (M,), generator=g)
    ids[torch.rand(M, generator=g) < 0.2] = 1
    pos = torch.randint(0, P, (M,), generator=g)
    tt = torch.randint(0, Tt, (M,), generator=g)
    ip = torch.randint(0, I, (M,), generator=g)
    lw = 1 + 0.1 * torch.randn(D, generator=g)
    lb = 0.1 * torch.randn(D, generator=g)
    dh = torch.randn(M, D, generator=g)
    x = (word[ids].double() + pe[pos].double() + te[tt].double() + ie[ip].double()).requires_grad_(True)
    w64, b64 = lw.double().requires_grad_(True), lb.double().requires_grad_(True)
    F.layer_norm(x, (D,), w64, b64, 1e-12).backward(dh.double())
    args = [t.to(dev) for t in (ids, pos, tt, ip, word, pe, te, ie, lw)]
    dx, dw, db = ops.embed_ln_bwd(*args, 1e-12, dh.to(dev))
    for got, ref in ((dx, x.grad), (dw, w64.grad), (db, b64.grad)):
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= 1e-5 * float(ref.abs().max()) + 1e-6, err
    dx2, dw2, db2 = ops.embed_ln_bwd(*args, 1e-12, dh.to(dev))
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)
    if D % 64:
        return  # the forward kernel (rf_embed_ln_fwd) takes widths in multiples of 64
    grads = {}
    for hip in (True, False):
        old, T.EMBED_BWD_HIP = T.EMBED_BWD_HIP, hip
        try:
            tabs = [t.to(dev).requires_grad_(True) for t in (word, pe, te, ie, lw, lb)]
            h = T._EmbedLN.apply(*args[:4], *tabs, 1e-12, 1)
            h.backward(dh.to(dev))
            grads[hip] = [t.grad for t in tabs]
        finally:
            T.EMBED_BWD_HIP = old
    for a, b in zip(grads[True], grads[False]):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-6
    assert float(grads[True][0][1].abs().max()) == 0.0 and float(grads[True][1][1].abs().max()) == 0.0


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_weight_pack_matches_torch_casts(dev, dt):
    """rf_pack_weights (ops.WeightPack): row-major compute-dtype copies and transposed copies of fp32
    sources, three sources stacked into one destination (the fused q|k|v weight), the first rows of
    the transposed copy scaled after rounding (round(round(w) * s), the q-column scale), ragged shapes
    (not multiples of 64), a source view with a row stride, a transposed-only and a plain-only entry:
    bit-identical to torch's .to(dt) / .t() / the scaled clone; refresh() re-reads updated sources."""
    g = torch.Generator(device="cpu").manual_seed(5)
    q, k, v = (torch.randn(200, 136, generator=g).to(dev) for _ in range(3))
    big = torch.randn(70, 300, generator=g).to(dev)
    view = big[:, 20:220]                       # lda 300
    w5 = torch.randn(64, 64, generator=g).to(dev)
    w6 = torch.randn(33, 100, generator=g).to(dev)
    qb, qt = torch.empty(600, 136, dtype=dt, device=dev), torch.empty(136, 600, dtype=dt, device=dev)
    vb, vt = torch.empty(70, 200, dtype=dt, device=dev), torch.empty(200, 70, dtype=dt, device=dev)
    t5 = torch.empty(64, 64, dtype=dt, device=dev)
    b6 = torch.empty(33, 100, dtype=dt, device=dev)
    s = 0.125
    pack = ops.WeightPack([dict(src=q, dst=(qb, 0), dstT=(qt, 0), scale_n=200, t_scale=s),
                           dict(src=k, dst=(qb, 200), dstT=(qt, 200)), dict(src=v, dst=(qb, 400), dstT=(qt, 400)),
                           dict(src=view, dst=(vb, 0), dstT=(vt, 0), scale_n=17, t_scale=0.3),
                           dict(src=w5, dstT=(t5, 0)), dict(src=w6, dst=(b6, 0))], dt)
    for rnd in range(2):
        pack.refresh()
        cat = torch.cat([q, k, v]).to(dt)
        assert torch.equal(qb, cat)
        ref_t = cat.clone()
        ref_t[:200] *= s
        assert torch.equal(qt, ref_t.t())
        vr = view.to(dt)
        assert torch.equal(vb, vr)
        vrt = vr.clone()
        vrt[:17] = (vrt[:17].float() * 0.3).to(dt)
        assert torch.equal(vt, vrt.t())
        assert torch.equal(t5, w5.to(dt).t())
        assert torch.equal(b6, w6.to(dt))
        with torch.no_grad():
            for w in (q, k, v, big, w5, w6):
                w.mul_(1.5)
    with pytest.raises(ValueError):
        ops.WeightPack([dict(src=q.t(), dst=(qb, 0))], dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (8192, 768, 3072), (4100, 2312, 768), (65536, 768, 768),
                                   (300, 520, 128), (70000, 2304, 768), (2048, 256, 192)])
def test_gemm_eight_wave_kernel(dev, dt, M, N, K):
    """The eight-wave ping-pong kernel (k_gemm_w8, knob gemm_w8; two waves per SIMD, one computing while its
    partner loads) for its epilogues (none, bias with a q-column scale, GELU): against fp32 torch on the same
    16-bit operands, and bit-identical to the four-wave kernel (the same MFMA sequence per accumulator and the
    same epilogue arithmetic), including ragged M / N edges (4100 x 2312, 300 x 520), a grid of fewer tiles
    than CUs (300 x 520), several tiles per CU (70000 x 2304) and the shortest K (128 / 192: 2 / 3 K-tiles)."""
    a = _rand((M, K), dev, dt, 0.5, seed=191)
    w = _rand((N, K), dev, dt, 0.05, seed=192)
    b = _rand((N,), dev, torch.float32, seed=193)
    prod = a.float() @ w.float().t()
    sc = N // 3 // 16 * 16
    tol = 4e-3 if dt == torch.float16 else 2e-2

    def rel(x, ref):
        return float((x.float() - ref).abs().max()) / max(1.0, float(ref.abs().max()))

    def run(knob):
        old = _lib.set_knob("gemm_w8", knob)
        try:
            return (ops.gemm(a, w, None, ops.RF_EPI_NONE),
                    ops.gemm(a, w, b, ops.RF_EPI_BIAS, scale_cols=sc, col_scale=0.125),
                    ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU))
        finally:
            _lib.set_knob("gemm_w8", old)

    none8, bias8, gelu8 = run(1)
    assert rel(none8, prod) <= tol
    ref = prod + b
    ref[:, :sc] *= 0.125
    assert rel(bias8, ref) <= tol
    assert rel(gelu8, F.gelu(prod + b)) <= tol
    none4, bias4, gelu4 = run(0)
    assert torch.equal(none8, none4)
    if dt == torch.bfloat16:
        assert torch.equal(bias8, bias4)
        assert torch.equal(gelu8, gelu4)
    else:
        # fp16: hipcc fuses the four-wave kernel's bias FMA and fp16 rounding into v_fma_mix on some values
        # (one rounding instead of fp32 then fp16): at most one fp16 ulp apart, and equal elsewhere
        for x8, x4 in ((bias8, bias4), (gelu8, gelu4)):
            d = (x8.float() - x4.float()).abs()
            ulp = torch.maximum(x4.float().abs(), torch.full_like(d, 2.0 ** -14)) * 2.0 ** -10
            assert bool((d <= ulp).all())
            assert float((d > 0).float().mean()) < 0.02
    # strided operand / output views (the q|k|v column slices the encoder hands over)
    wide = torch.zeros(M, N + 64, device=dev, dtype=dt)
    old = _lib.set_knob("gemm_w8", 1)
    try:
        ops.gemm(a, w, b, ops.RF_EPI_BIAS, scale_cols=sc, col_scale=0.125, out=wide[:, 16:16 + N])
    finally:
        _lib.set_knob("gemm_w8", old)
    assert torch.equal(wide[:, 16:16 + N], bias8)
    assert not wide[:, :16].any() and not wide[:, 16 + N:].any()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (8192, 768, 3072), (4100, 2312, 768), (65536, 768, 768),
                                   (300, 520, 128), (70000, 2304, 768), (2048, 256, 192)])
def test_gemm_split_plane_kernel(dev, dt, M, N, K):
    """The four-wave kernel on k-step-split LDS planes (k_gemm_w4p, knob gemm_w4p: the operand DMA spread
    over both phases of a K-tile) for its epilogues (none, bias with a q-column scale, GELU): against fp32
    torch on the same 16-bit operands and bit-identical to k_gemm_w4 (same MFMA sequence, same epilogue code),
    ragged M / N edges, fewer tiles than CUs, several tiles per CU, the shortest K (2 / 3 K-tiles)."""
    a = _rand((M, K), dev, dt, 0.5, seed=291)
    w = _rand((N, K), dev, dt, 0.05, seed=292)
    b = _rand((N,), dev, torch.float32, seed=293)
    prod = a.float() @ w.float().t()
    sc = N // 3 // 16 * 16
    tol = 4e-3 if dt == torch.float16 else 2e-2

    def rel(x, ref):
        return float((x.float() - ref).abs().max()) / max(1.0, float(ref.abs().max()))

    def run(knob):
        old = _lib.set_knob("gemm_w4p", knob)
        try:
            return (ops.gemm(a, w, None, ops.RF_EPI_NONE),
                    ops.gemm(a, w, b, ops.RF_EPI_BIAS, scale_cols=sc, col_scale=0.125),
                    ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU))
        finally:
            _lib.set_knob("gemm_w4p", old)

    outs = run(1)
    assert rel(outs[0], prod) <= tol
    ref = prod + b
    ref[:, :sc] *= 0.125
    assert rel(outs[1], ref) <= tol
    assert rel(outs[2], F.gelu(prod + b)) <= tol
    for x, y in zip(outs, run(0)):
        if dt == torch.bfloat16:
            assert torch.equal(x, y)
        else:  # fp16: at most one ulp where hipcc fuses a bias FMA with the fp16 rounding differently
            d = (x.float() - y.float()).abs()
            assert bool((d <= torch.maximum(y.float().abs(), torch.full_like(d, 2.0 ** -14)) * 2.0 ** -10).all())


@pytest.mark.parametrize("mfma32", [0, 1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (8192, 768, 3072), (4100, 2312, 768), (65536, 768, 768)])
def test_gemm_four_wave_kernels_all_epilogues(dev, mfma32, dt, M, N, K):
    """Both four-wave 256x256 kernels — k_gemm_w4 (v_mfma_f32_16x16x32) and k_gemm_w32
    (v_mfma_f32_32x32x16, knob gemm_mfma32) — for every epilogue the encoder and its backward use
    (none, bias with a q-column scale, GELU, GELU + pre-activation, the GELU-backward DGELU, fp32
    output, cosine scores), including ragged M / N edges (4100 x 2312), against fp32 torch on the
    same 16-bit operands."""
    old = _lib.set_knob("gemm_mfma32", mfma32)
    old192 = _lib.set_knob("gemm_n192", 0)  # the 256 x 256 tiles here (the 192-column one: its own test)
    try:
        a = _rand((M, K), dev, dt, 0.5, seed=91)
        w = _rand((N, K), dev, dt, 0.05, seed=92)
        b = _rand((N,), dev, torch.float32, seed=93)
        prod = a.float() @ w.float().t()
        sc = N // 3 // 16 * 16
        tol = 4e-3 if dt == torch.float16 else 2e-2

        def rel(x, ref):
            return float((x.float() - ref).abs().max()) / max(1.0, float(ref.abs().max()))

        out = ops.gemm(a, w, None, ops.RF_EPI_NONE)
        assert rel(out, prod) <= tol
        ref = prod + b
        ref[:, :sc] *= 0.125
        out = ops.gemm(a, w, b, ops.RF_EPI_BIAS, scale_cols=sc, col_scale=0.125)
        assert rel(out, ref) <= tol
        out32 = ops.gemm(a, w, b, ops.RF_EPI_BIAS, out_f32=True)
        assert float((out32 - (prod + b)).abs().max()) <= 1e-3 * max(1.0, float(prod.abs().max()))
        gl = ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU)
        assert rel(gl, F.gelu(prod + b)) <= tol
        z = torch.full((M, N), 7.0, device=dev, dtype=dt)
        u = ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
        assert torch.equal(u, gl)
        assert torch.equal(z, ops.gemm(a, w, b, ops.RF_EPI_BIAS))
        zz = _rand((M, N), dev, dt, 2.0, seed=94)
        dg = ops.gemm(a, w, None, ops.RF_EPI_DGELU, resid=zz)
        ref = torch.ops.aten.gelu_backward(prod, zz.float())
        assert float((dg.float() - ref).abs().max()) <= 1e-2 * max(float(ref.abs().max()), 1e-6)
        ra = (1.0 / a.float().norm(dim=-1).clamp_min(1e-8)).contiguous()
        rw = (1.0 / w.float().norm(dim=-1).clamp_min(1e-8)).contiguous()
        cs = ops.cos_scores(a, w, 20.0, z_rnorm=ra, items_rnorm=rw)
        ref = F.normalize(a.float(), dim=-1) @ F.normalize(w.float(), dim=-1).t() * 20.0
        assert float((cs - ref).abs().max()) <= 2e-2
    finally:
        _lib.set_knob("gemm_mfma32", old)
        _lib.set_knob("gemm_n192", old192)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (16384, 768, 3072), (16347, 760, 768), (10000, 1000, 1024)])
def test_gemm_192_column_tiles(dev, dt, M, N, K):
    """The four-wave kernel on 256 x 192 tiles (knob gemm_n192, off by default: the N = 768 products at the training
    batch, 256 tiles instead of 192 of 256^2) computes every output element with the same MFMA sequence
    as the 256 x 256 tile: bit-identical to it for EPI_NONE, EPI_BIAS and the 16-bit-residual
    EPI_BIAS_RESID in bf16 (fp16 with a bias: within 1 ulp, see below), ragged M / N edges included,
    and within the 16-bit tolerance of fp32 torch. The profiler shows which kernel ran."""
    from torch.profiler import ProfilerActivity, profile
    a = _rand((M, K), dev, dt, 0.5, seed=71)
    w = _rand((N, K), dev, dt, 0.05, seed=72)
    b = _rand((N,), dev, torch.float32, seed=73)
    r = _rand((M, N), dev, dt, 1.0, seed=74)  # a 16-bit residual (the training dA GEMM's mailbox form)
    res = {}
    old = _lib.set_knob("gemm_n192", 0)
    try:
        for knob in (0, 1):
            _lib.set_knob("gemm_n192", knob)
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                res[knob] = (ops.gemm(a, w, None, ops.RF_EPI_NONE), ops.gemm(a, w, b, ops.RF_EPI_BIAS),
                             ops.gemm(a, w, b, ops.RF_EPI_BIAS_RESID, resid=r))
                torch.cuda.synchronize()
            names = [e.name for e in prof.events() if "k_gemm_w4" in e.name]
            if names:  # the 192-column instantiation carries NJ = 6 in its mangled name
                assert any("Li6EEEvi" in n for n in names) == (knob == 1), names
    finally:
        _lib.set_knob("gemm_n192", old)
    for n, (x, y) in enumerate(zip(res[0], res[1])):
        if dt == torch.bfloat16 or n == 0:
            assert torch.equal(x, y)
        else:
            # fp16 with a bias: the 256-column kernel's fp32 bias add and fp16 rounding are partly fused
            # by hipcc into one v_fma_mix (one rounding), the 192-column kernel rounds twice (fp32, then
            # fp16) like the other epilogues: at most 1 ulp apart, in ~1e-5 of the outputs
            d = (x.float() - y.float()).abs()
            ulp = torch.finfo(torch.float16).eps * torch.maximum(x.float().abs(), y.float().abs())
            assert bool((d <= ulp).all()), float((d / ulp.clamp_min(1e-30)).max())
            assert int((x != y).sum()) <= 1e-4 * x.numel()
    prod = a.float() @ w.float().t()
    tol = 4e-3 if dt == torch.float16 else 2e-2
    for x, ref in zip(res[1], (prod, prod + b, prod + b + r.float())):
        assert float((x.float() - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,N,C", [(16, 10000, None), (16, 10000, 1001), (3, 700, None), (5, 200, 37), (40, 333, None)])
def test_cos_scores_bwd_matches_autograd(dev, dt, B, N, C):
    """rf_cos_score_bwd (the training scoring head's dL/dz, Similarity models.py:358-369 under the
    CrossEntropyLoss of :583-599) against autograd through fp32 torch normalize + matmul / gather,
    for the full catalog (C None: rows sharing the table, B > 16 in row groups) and sampled
    candidates (cand (B, C) incl. repeats), with a CE-shaped upstream gradient."""
    from recformer_amd import train
    g = torch.Generator(device=dev).manual_seed(B * 7 + N)
    z = torch.randn(B, 768, device=dev, generator=g).to(dt)
    items = torch.randn(N, 768, device=dev, generator=g).to(dt)
    items[3] *= 1e-3
    inv_t = 20.0
    cand = torch.randint(0, N, (B, C), device=dev, generator=g) if C else None
    labels = torch.randint(0, C or N, (B,), device=dev, generator=g)
    rt = ops.row_inv_norm(items)
    zf = z.float().requires_grad_(True)
    itf = items.float()
    zn = zf / zf.norm(dim=-1, keepdim=True).clamp_min(1e-8)
    itn = itf / itf.norm(dim=-1, keepdim=True).clamp_min(1e-8)
    ref_s = zn @ itn.t() * inv_t if cand is None else torch.einsum("bd,bcd->bc", zn, itn[cand]) * inv_t
    F.cross_entropy(ref_s, labels).backward()
    zh = z.float().contiguous().requires_grad_(True)
    if dt == torch.float32:
        s = train.cos_scores_train(zh, items, rt, inv_t, cand)
        loss = train.cross_entropy_train(s, labels)
        loss.backward()
        assert float((s - ref_s).abs().max()) <= 1e-4 * inv_t
        dz = zh.grad
    else:
        s = ref_s.detach()
        gs = torch.softmax(s, -1)
        gs[torch.arange(B), labels] -= 1
        gs /= B
        dz = ops.cos_scores_bwd(z, items, gs.contiguous(), s.contiguous(), inv_t, ops.row_inv_norm(z), rt, cand)
    err = float((dz - zf.grad).abs().max())
    assert err <= 2e-3 * float(zf.grad.abs().max()) + 1e-7, err
    if dt != torch.float32:  # fixed-order sums: bit-identical on a repeat
        again = ops.cos_scores_bwd(z, items, gs.contiguous(), s.contiguous(), inv_t, ops.row_inv_norm(z), rt, cand)
        assert torch.equal(dz, again)


@pytest.mark.parametrize("skinny", [0, 1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(64, 3072, 768), (16, 768, 3072), (1, 2304, 768), (40, 768, 768)])
def test_gemm_few_rows_all_epilogues(dev, skinny, dt, M, N, K):
    """GEMMs with M <= 64 rows (the CLS-only last layer, the global query rows): k_gemm_skinny (knob
    gemm_skinny, K split over the four waves and summed in LDS) and the 128 x 128 kernel, for the
    epilogues those rows use, against fp32 torch on the same 16-bit operands."""
    old = _lib.set_knob("gemm_skinny", skinny)
    try:
        a = _rand((M, K), dev, dt, 0.5, seed=71)
        w = _rand((N, K), dev, dt, 0.05, seed=72)
        b = _rand((N,), dev, torch.float32, seed=73)
        prod = a.float() @ w.float().t()
        tol = 4e-3 if dt == torch.float16 else 2e-2

        def rel(x, ref):
            return float((x.float() - ref).abs().max()) / max(1.0, float(ref.abs().max()))

        assert rel(ops.gemm(a, w, None, ops.RF_EPI_NONE), prod) <= tol
        sc = N // 3 // 16 * 16
        ref = prod + b
        ref[:, :sc] *= 0.125
        assert rel(ops.gemm(a, w, b, ops.RF_EPI_BIAS, scale_cols=sc, col_scale=0.125), ref) <= tol
        out32 = ops.gemm(a, w, b, ops.RF_EPI_BIAS, out_f32=True)
        assert float((out32 - (prod + b)).abs().max()) <= 1e-3 * max(1.0, float(prod.abs().max()))
        gl = ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU)
        assert rel(gl, F.gelu(prod + b)) <= tol
        z = torch.empty(M, N, device=dev, dtype=dt)
        u = ops.gemm(a, w, b, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
        assert torch.equal(u, gl)
        assert rel(z, prod + b) <= tol
        zz = _rand((M, N), dev, dt, 2.0, seed=74)
        dg = ops.gemm(a, w, None, ops.RF_EPI_DGELU, resid=zz)
        ref = torch.ops.aten.gelu_backward(prod, zz.float())
        assert float((dg.float() - ref).abs().max()) <= 1e-2 * max(float(ref.abs().max()), 1e-6)
    finally:
        _lib.set_knob("gemm_skinny", old)
