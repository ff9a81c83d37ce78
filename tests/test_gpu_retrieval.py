"""C5 retrieval (rf_retrieval.hip, recformer_amd.ranker): the fused score + rank + top-k kernels
against the Ranker restated from utils.py:76-108 (oracle.restatement.ranker_metrics, pinned to the
real Ranker's outputs by tests/golden/ranker.npz) on the scores of the same kernel written densely
(bit-identical by construction: same MFMA chain, same epilogue expression), and the top-k against
a full sort of those scores (ties by lower item id)."""
import pytest
import torch

from oracle import restatement as R
from recformer_amd import _lib, ops
from recformer_amd.ranker import (CatalogShard, _score_rank, combine_shards, label_scores, merge_topk, rank_catalog,
                                  shard_rank)

pytestmark = pytest.mark.gpu
KS = [1, 5, 10, 20, 50]


def _dense_scores(q, shard, s_label, temp, chunk=8192):
    """(B, N) fp32 scores from rf_score_rank's dense mode, chunk by chunk."""
    B, N = q.shape[0], shard.n
    qn = ops.row_inv_norm(q)
    nt = _lib.load().rf_score_rank_tiles(chunk)
    pc = torch.empty(nt, B, dtype=torch.int32, device=q.device)
    ps = torch.empty(nt, B, dtype=torch.float32, device=q.device)
    out = torch.empty(B, N, dtype=torch.float32, device=q.device)
    buf = torch.empty(B, chunk, dtype=torch.float32, device=q.device)
    for off in range(0, N, chunk):
        n = min(chunk, N - off)
        _score_rank(q, qn, shard, s_label, 1.0 / temp, 0, off, n, pc, ps, 0, dense=buf)
        out[:, off:off + n] = buf[:, :n]
    return out


def _case(dev, dt, B, N, seed, dup=True, cluster=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    q = torch.randn(B, 768, device=dev, generator=g)
    items = torch.randn(N, 768, device=dev, generator=g)
    labels = torch.randint(0, N, (B,), device=dev, generator=g)
    labels[::3] = N - 1 - torch.arange(len(labels[::3]), device=dev) % 7  # last (partial) tile
    if dup:  # exact duplicates of some label items elsewhere (ties with the label score)
        d = labels[: min(B, 16)]
        items[(d + N // 2) % N] = items[d]
    if cluster:  # `cluster` near-copies of query 0 inside one 256-item tile: its candidate slots overflow
        items[256:256 + cluster] = q[0] + 1e-3 * torch.randn(cluster, 768, device=dev, generator=g)
    return q.to(dt), items.to(dt), labels


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_label_scores_bit_identical_to_ranking_kernel(dev, dt):
    q, items, labels = _case(dev, dt, 77, 5003, 1)
    shard = CatalogShard(items)
    sl = label_scores(q, shard, labels, 0.05)
    dense = _dense_scores(q, shard, sl, 0.05)
    assert torch.equal(sl, dense.gather(1, labels[:, None]).squeeze(1))
    # labels outside a shard contribute exactly 0
    half = CatalogShard(items[:2500], base=0)
    s_half = label_scores(q, half, labels, 0.05)
    assert torch.equal(s_half[labels >= 2500], torch.zeros_like(s_half[labels >= 2500]))


@pytest.mark.parametrize("growth", [2, 8])
@pytest.mark.parametrize("dt,B,N,cluster", [(torch.bfloat16, 37, 20011, 0), (torch.float16, 300, 33000, 0),
                                            (torch.bfloat16, 64, 12000, 200)])
def test_shard_rank_matches_restated_ranker_and_sort(dev, monkeypatch, dt, B, N, cluster, growth):
    """Strict ranks, valid lengths and the Ranker metrics equal the restated Ranker on the same
    scores; the top-50 equals a full stable sort; a row whose candidate slots overflow (cluster of
    near-copies in one tile) is re-ranked exactly. growth: the candidate chunks' growth factor
    (ranker.TOPK_GROWTH; 2 = each chunk as large as everything before it)."""
    import recformer_amd.ranker as RK
    monkeypatch.setattr(RK, "TOPK_GROWTH", growth)
    q, items, labels = _case(dev, dt, B, N, B + N, cluster=cluster)
    shard = CatalogShard(items)
    sl = label_scores(q, shard, labels, 0.05)
    parts = shard_rank(q, shard, sl, 0.05, k=50)
    dense = _dense_scores(q, shard, sl, 0.05)
    ref_rank = (dense > sl[:, None]).sum(1)
    assert torch.equal(parts["gt"].long(), ref_rank)
    assert torch.equal(parts["valid"].long(), torch.full_like(ref_rank, N))
    ref = R.ranker_metrics(dense.cpu(), labels.cpu(), KS)
    loss = float((torch.log(parts["sexp"]) + parts["shift"] - sl).mean())
    from recformer_amd.ranker import _metrics
    got = _metrics(parts["gt"], parts["valid"], loss, KS)
    for a, b in zip(got[:-1], ref[:-1]):
        assert a == pytest.approx(b, abs=1e-6)
    assert got[-1] == pytest.approx(ref[-1], rel=1e-4)
    ids = torch.arange(N, device=dev, dtype=torch.int32).expand(B, N)
    rv, ri = merge_topk(dense, ids, 50)
    assert torch.equal(parts["topv"], rv)
    assert torch.equal(parts["topi"], ri)


@pytest.mark.parametrize("k", [128, 256])
def test_shard_rank_large_k_few_overflows(dev, k):
    """At large k the chunk growth is capped (ranker.growth_for: k * (grow - 1) <= cap / 2), so
    the candidate lists do not overflow into the dense re-rank for most rows (advisor r05: at
    k = 256 a growth of 8 overflowed nearly every row); the top-k still equals a full sort."""
    import recformer_amd.ranker as RK
    assert RK.growth_for(50) == RK.TOPK_GROWTH and RK.growth_for(256) == 3 and RK.growth_for(128) == 5
    B, N = 256, 60000
    q, items, labels = _case(dev, torch.bfloat16, B, N, B + N)
    shard = CatalogShard(items)
    sl = label_scores(q, shard, labels, 0.05)
    parts = shard_rank(q, shard, sl, 0.05, k=k)
    assert parts["overflow"] <= B // 20, parts["overflow"]
    dense = _dense_scores(q, shard, sl, 0.05)
    ids = torch.arange(N, device=dev, dtype=torch.int32).expand(B, N)
    rv, ri = merge_topk(dense, ids, k)
    assert torch.equal(parts["topv"], rv)
    assert torch.equal(parts["topi"], ri)


def test_two_shards_combine_to_one(dev):
    """The catalog split in two shards (global ids), label scores summed, counts summed and the
    shards' top-k merged (what combine_shards does across ranks) equals the single-shard result."""
    q, items, labels = _case(dev, torch.float16, 129, 30000, 5)
    whole = CatalogShard(items)
    sl = label_scores(q, whole, labels, 0.05)
    one = shard_rank(q, whole, sl, 0.05, k=50)
    a, b = CatalogShard(items[:17000], 0), CatalogShard(items[17000:], 17000)
    sl2 = label_scores(q, a, labels, 0.05) + label_scores(q, b, labels, 0.05)
    assert torch.equal(sl2, sl)
    pa, pb = shard_rank(q, a, sl2, 0.05, k=50), shard_rank(q, b, sl2, 0.05, k=50)
    assert torch.equal(pa["gt"] + pb["gt"], one["gt"])
    v, i = merge_topk(torch.cat([pa["topv"], pb["topv"]], 1), torch.cat([pa["topi"], pb["topi"]], 1), 50)
    assert torch.equal(v, one["topv"]) and torch.equal(i, one["topi"])
    single = combine_shards(one, 50)  # one rank: identity
    assert single["topi"] is one["topi"]


def test_rank_catalog_large_fp16(dev):
    """N >= 262k: rank_catalog (counts-only kernel mode) vs the restated Ranker
    on the dense scores of the same kernel; fp16 operands."""
    q, items, labels = _case(dev, torch.float16, 512, 262144 + 37, 9)
    shard = CatalogShard(items)
    sl = label_scores(q, shard, labels, 0.05)
    dense = _dense_scores(q, shard, sl, 0.05)
    ref = R.ranker_metrics(dense.cpu(), labels.cpu(), KS)
    got = rank_catalog(q, items, labels, KS, 0.05)
    for x, y in zip(got[:-1], ref[:-1]):
        assert x == pytest.approx(y, abs=1e-6)
    assert got[-1] == pytest.approx(ref[-1], rel=1e-4)


def _fp32_scores(q, items, temp, chunk=65536):
    """(B, N) cos(q, items) / temp in fp32 from the 16-bit values (plain torch, no kernel of ours)."""
    qf = q.float()
    qf = qf / qf.norm(dim=1, keepdim=True).clamp_min(1e-8)
    out = torch.empty(q.shape[0], items.shape[0], dtype=torch.float32, device=q.device)
    for off in range(0, items.shape[0], chunk):
        it = items[off:off + chunk].float()
        it = it / it.norm(dim=1, keepdim=True).clamp_min(1e-8)
        out[:, off:off + chunk] = (qf @ it.t()) / temp
    return out


@pytest.mark.parametrize("dt,B,N", [(torch.float16, 64, 33000), (torch.float16, 64, 262144 + 37),
                                    (torch.bfloat16, 64, 262144 + 37), (torch.float16, 32, 1000000)])
def test_retrieval_scores_and_topk_vs_fp32_torch(dev, dt, B, N):
    """C5 against an independent fp32 reference: the fused kernel's scores (its dense
    mode, the same MFMA chain and epilogue the ranking pass uses) within 2e-2 of torch's fp32
    cos / temp on the same 16-bit values (temp 0.05, |score| <= 20), at 33k, 262k and 1M items;
    the strict rank counts within the rows' near-tie band of that reference; and retrieve()'s
    top-50 equal to an fp32 sort of the catalog except where the two scores of a swapped pair are
    within that tolerance (near-ties), with the 50th score within tolerance."""
    from recformer_amd.ranker import retrieve
    tol = 2e-2
    q, items, labels = _case(dev, dt, B, N, 3 * B + N, dup=False)
    shard = CatalogShard(items)
    sl = label_scores(q, shard, labels, 0.05)
    ref = _fp32_scores(q, items, 0.05)
    dense = _dense_scores(q, shard, sl, 0.05, chunk=65536)
    err = float((dense - ref).abs().max())
    assert err <= tol, err
    # ranks: every item the reference puts clearly above the label is counted, none clearly below
    parts = shard_rank(q, shard, sl, 0.05, k=0)
    ref_sl = ref.gather(1, labels[:, None])
    lo = (ref > ref_sl + 2 * tol).sum(1)
    hi = (ref > ref_sl - 2 * tol).sum(1)
    gt = parts["gt"].long()
    assert bool(((gt >= lo) & (gt <= hi)).all())
    # top-50 vs an fp32 sort
    _, topv, topi = retrieve(q, shard, labels, KS, 0.05, k=50)
    rv, ri = torch.sort(ref, dim=1, descending=True)
    rv, ri = rv[:, :50], ri[:, :50]
    assert float((topv - rv).abs().max()) <= tol
    got_ref = ref.gather(1, topi.long())  # the reference's scores of the items we returned
    # any item we return scores, in the reference, within tol of the reference's 50th score or above
    assert bool((got_ref >= rv[:, 49:50] - 2 * tol).all())
    # and the sets agree on every item the reference ranks clearly inside the top 50
    clear = rv > (rv[:, 49:50] + 2 * tol)
    for b in range(B):
        want = set(ri[b][clear[b]].tolist())
        assert want <= set(topi[b].tolist()), b


@pytest.mark.parametrize("w32", [0, 1])
@pytest.mark.parametrize("dt,B,N,cluster", [(torch.bfloat16, 300, 70001, 0), (torch.float16, 64, 12000, 200),
                                            (torch.float16, 513, 33000, 0)])
def test_rank_kernels_both_paths(dev, w32, dt, B, N, cluster):
    """The 32x32x16 four-wave score + rank kernel (knob rank_w32: items as the MFMA A operand, per-query
    counts as in-lane sums, candidates through per-lane slots) and the 16x16x32 kernel: on each path
    the label scores are bit-identical to the path's dense scores, the strict ranks / valid counts equal
    a count over those scores, and the top-50 equals a full sort of them (overflowing rows re-ranked);
    the two paths' scores agree to fp32 rounding."""
    old = _lib.set_knob("rank_w32", w32)
    try:
        q, items, labels = _case(dev, dt, B, N, B * 7 + N, cluster=cluster)
        shard = CatalogShard(items)
        sl = label_scores(q, shard, labels, 0.05)
        dense = _dense_scores(q, shard, sl, 0.05)
        assert torch.equal(sl, dense.gather(1, labels[:, None]).squeeze(1))
        parts = shard_rank(q, shard, sl, 0.05, k=50)
        assert torch.equal(parts["gt"].long(), (dense > sl[:, None]).sum(1))
        assert torch.equal(parts["valid"].long(), torch.full((B,), N, dtype=torch.long, device=dev))
        ref_se = torch.exp(dense.double() - parts["shift"]).sum(1)
        assert torch.allclose(parts["sexp"].double(), ref_se, rtol=1e-4)
        ids = torch.arange(N, device=dev, dtype=torch.int32).expand(B, N)
        rv, ri = merge_topk(dense, ids, 50)
        assert torch.equal(parts["topv"], rv)
        assert torch.equal(parts["topi"], ri)
        _lib.set_knob("rank_w32", 1 - w32)
        other = _dense_scores(q, shard, label_scores(q, shard, labels, 0.05), 0.05)
        assert float((other - dense).abs().max()) <= 1e-4 * 20
    finally:
        _lib.set_knob("rank_w32", old)
