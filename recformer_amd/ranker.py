"""Ranker — drop-in for the reference's evaluation metrics (utils.py:76-108; callers
finetune.py:70-92, evaluate_seq.py:35-52).

forward(scores, labels) -> [NDCG@k, Recall@k for k in ks] + [MRR, AUC, loss], Python floats as
the reference returns them. The per-row counts (rank = #{n: s_n > s_label}, strict;
valid_length = #{n: s_n > -MAX_VAL}) come from rf_rank_accum and the cross entropy from
rf_cross_entropy_fwd; only the final means are torch reductions. Works on score blocks of any
width (the counts accumulate), so a catalog can also be ranked block by block.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from . import _lib, ops

MAX_VAL = 1e4  # utils.py:5


def rank_counts(scores: torch.Tensor, labels: torch.Tensor, max_val: float = MAX_VAL):
    """(rank, valid_length) per row, int32, on the HIP kernel."""
    lib = _lib.load()
    if not scores.is_cuda:
        raise _lib.RecformerHipError("Ranker needs ROCm device tensors (no CPU fallback)")
    s = scores.float()
    if s.stride(1) != 1:
        s = s.contiguous()
    B = s.shape[0]
    lab = labels.reshape(-1).long()
    s_label = s[torch.arange(B, device=s.device), lab].contiguous()
    gt = torch.zeros(B, dtype=torch.int32, device=s.device)
    valid = torch.zeros(B, dtype=torch.int32, device=s.device)
    _lib.check(lib.rf_rank_accum(B, s.shape[1], s.data_ptr(), s.stride(0), s_label.data_ptr(), float(max_val),
                                 0.0, gt.data_ptr(), valid.data_ptr(), None,
                                 torch.cuda.current_stream(s.device).cuda_stream), "rf_rank_accum")
    return gt, valid


class Ranker(nn.Module):
    """utils.py:76-108 on the HIP path."""

    def __init__(self, metrics_ks: Sequence[int]):
        super().__init__()
        self.ks = list(metrics_ks)

    def forward(self, scores: torch.Tensor, labels: torch.Tensor) -> List[float]:
        labels = labels.squeeze()
        try:
            loss = float(ops.cross_entropy(scores.float(), labels.reshape(-1)))
        except Exception:  # utils.py:86-90 reports and continues with 0
            print(scores.size())
            print(labels.size())
            loss = 0.0
        gt, valid = rank_counts(scores, labels.reshape(-1))
        return _metrics(gt, valid, loss, self.ks)


def _metrics(gt: torch.Tensor, valid: torch.Tensor, loss: float, metrics_ks: Sequence[int]) -> List[float]:
    """The Ranker's list (utils.py:95-108) from per-row strict ranks and valid lengths."""
    rank = gt.float()
    res = []
    for k in metrics_ks:
        indicator = (rank < k).float()
        res.append(((1 / torch.log2(rank + 2)) * indicator).mean().item())  # ndcg@k
        res.append(indicator.mean().item())  # hr@k
    res.append((1 / (rank + 1)).mean().item())  # MRR
    res.append((1 - (rank / valid.float())).mean().item())  # AUC
    return res + [loss]


# ---- C5 retrieval: catalog shards, fused score + rank + top-k (rf_retrieval.hip) -----------------
TOPK_SAMPLE = 2048  # dense seed block that sets each row's first candidate threshold
TOPK_CAP = 1024     # candidate list per row and chunk
TOPK_MAX_K = 256    # rf_topk_* limits (rf_retrieval.hip TK_KMAX, TK_DENSE_MAX)
TOPK_MAX_SAMPLE = 2048
TILE_CAND_CAP = 32  # rf_retrieval.hip RK_TCAP: candidates staged per (row, 256-column tile)
# column chunks after the seed: each TOPK_GROWTH - 1 times the columns already seen (2: doubling). A larger
# factor means fewer launches and merges but a lower threshold relative to each chunk (about
# k * (TOPK_GROWTH - 1) candidates per row and chunk). 1M items x 4096 queries, top-50, 16x16x32 family:
# 9.27 / 9.11 / 9.05 ms at 2 / 4 / 8 (the 32x32x16 family 10.2-10.4 ms at any; gpurun_out/r05f/c5ab.log)
TOPK_GROWTH = 8


def growth_for(k: int, cap: int = TOPK_CAP) -> int:
    """Chunk growth factor for a top-k of k with `cap` candidate slots per row and chunk: TOPK_GROWTH,
    limited so the expected k * (grow - 1) candidates fill at most half the list (2 at the least)."""
    if k <= 0:
        return max(2, int(TOPK_GROWTH))
    return max(2, min(int(TOPK_GROWTH), 1 + cap // (2 * k)))


@contextlib.contextmanager
def _rank_family(topk: bool):
    """The rank kernel family for one self-contained ranking (label scores + rank counts from the same
    arithmetic, so the strict counts and exact ties stay the full-matrix Ranker's): the 32x32x16 loop
    for counts only (1M x 4096: 6.96 vs 7.89 ms), the 16x16x32 one with a top-k (round 6, both with the
    register top-k and the 32x32x16 candidate epilogue without spills: 125k 1.361 vs 1.456 ms, 1M 8.838
    vs 9.419 ms; profiles/r06/c5_family_ab.jsonl). label_scores / shard_rank called directly follow the
    knob rank_w32."""
    old = _lib.set_knob("rank_w32", 0 if topk else 1)
    try:
        yield
    finally:
        _lib.set_knob("rank_w32", old)


def _check_topk_args(k: int, sample: int, cap: int) -> None:
    if not 0 <= k <= TOPK_MAX_K:
        raise ValueError(f"top-k: k={k} must be in [0, {TOPK_MAX_K}]")
    if k > 0 and not k <= sample <= TOPK_MAX_SAMPLE:
        raise ValueError(f"top-k: sample={sample} must be in [k={k}, {TOPK_MAX_SAMPLE}]")
    if k > 0 and cap < 1:
        raise ValueError(f"top-k: cap={cap} must be positive")


class CatalogShard:
    """One GPU's shard of the item table for retrieval (the 1M-item catalog sharded
    over the GPUs of a node): items (N_s, d) in bf16 or fp16 with global ids base .. base + N_s - 1,
    and their inverse norms (Similarity's clamp, models.py:366) computed once."""

    def __init__(self, items: torch.Tensor, base: int = 0, rnorm: Optional[torch.Tensor] = None):
        if not items.is_cuda:
            raise _lib.RecformerHipError("CatalogShard needs a ROCm device tensor (no CPU fallback)")
        if items.dtype not in (torch.bfloat16, torch.float16):
            raise TypeError("CatalogShard: items must be bf16 or fp16")
        self.items = items.contiguous()
        self.base = int(base)
        self.rnorm = ops.row_inv_norm(self.items) if rnorm is None else rnorm.float().contiguous()

    @property
    def n(self) -> int:
        return self.items.shape[0]


def _check_q(queries: torch.Tensor, shard: CatalogShard) -> torch.Tensor:
    q = queries.contiguous()
    if q.dtype != shard.items.dtype or q.shape[1] != shard.items.shape[1]:
        raise ValueError("queries and catalog must share dtype and width")
    if q.shape[1] % 32 or q.data_ptr() % 16 or shard.items.data_ptr() % 16:
        raise ValueError("retrieval kernels need d % 32 == 0 and 16-B aligned rows")
    return q


def label_scores(queries: torch.Tensor, shard: CatalogShard, labels: torch.Tensor, temp: float,
                 q_rnorm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cos(q_b, E[label_b]) / temp for the labels inside this shard, 0 for the others (summed over
    the shards this is every row's label score, bit-identical to the ranking kernel's value)."""
    q = _check_q(queries, shard)
    qn = ops.row_inv_norm(q) if q_rnorm is None else q_rnorm
    lab = labels.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty(q.shape[0], dtype=torch.float32, device=q.device)
    _lib.check(_lib.load().rf_label_scores(ops.dtype_code(q.dtype), q.shape[0], q.shape[1], q.data_ptr(), q.stride(0),
                                           qn.data_ptr(), shard.items.data_ptr(), shard.items.stride(0),
                                           shard.rnorm.data_ptr(), shard.n, lab.data_ptr(), shard.base,
                                           float(1.0 / temp), out.data_ptr(), ops._stream(q)), "rf_label_scores")
    return out


def _score_rank(q, qn, shard, s_label, inv_t, mode, col0, ncols, part_cnt, part_sexp, tn0, dense=None, tau=None,
                cand=None, max_val=MAX_VAL):
    lib = _lib.load()
    cval, cidx, rcnt = cand if cand is not None else (None, None, None)
    capr = cval.shape[1] if cval is not None else 1
    p = ops._p
    _lib.check(lib.rf_score_rank(ops.dtype_code(q.dtype), mode, q.shape[0], q.shape[1], q.data_ptr(), q.stride(0),
                                 qn.data_ptr(), shard.items.data_ptr(), shard.items.stride(0), shard.rnorm.data_ptr(),
                                 col0, ncols, float(inv_t), s_label.data_ptr(), float(max_val), float(inv_t), p(tau),
                                 p(dense), dense.stride(0) if dense is not None else 0, p(cval), p(cidx), p(rcnt), capr,
                                 shard.base, part_cnt.data_ptr(), part_sexp.data_ptr(), tn0, ops._stream(q)),
               "rf_score_rank")


def _topk_dense(vals: torch.Tensor, k: int, idx: Optional[torch.Tensor] = None, idx_base: int = 0):
    B, n = vals.shape
    ov = torch.empty(B, k, dtype=torch.float32, device=vals.device)
    oi = torch.empty(B, k, dtype=torch.int32, device=vals.device)
    _lib.check(_lib.load().rf_topk_dense(B, n, vals.data_ptr(), vals.stride(0), ops._p(idx),
                                         idx.stride(0) if idx is not None else 0, idx_base, k, ov.data_ptr(),
                                         oi.data_ptr(), ops._stream(vals)), "rf_topk_dense")
    return ov, oi


def _dense_topk_rows(q, qn, shard, s_label, inv_t, k, col0, ncols, prev_v, prev_i, chunk=TOPK_SAMPLE):
    """Exact top-k of the rows of q over shard rows [col0, col0 + ncols) merged with their running
    top-k (prev_v, prev_i), densely chunk by chunk (the candidate-overflow path)."""
    B = q.shape[0]
    nt = _lib.load().rf_score_rank_tiles(chunk)
    pc = torch.empty(nt, B, dtype=torch.int32, device=q.device)
    ps = torch.empty(nt, B, dtype=torch.float32, device=q.device)
    dense = torch.empty(B, chunk, dtype=torch.float32, device=q.device)
    bv, bi = prev_v, prev_i
    for off in range(col0, col0 + ncols, chunk):
        n = min(chunk, col0 + ncols - off)
        _score_rank(q, qn, shard, s_label, inv_t, 0, off, n, pc, ps, 0, dense=dense)
        v, i = _topk_dense(dense[:, :n], k, idx_base=shard.base + off)
        bv, bi = _topk_dense(torch.cat([bv, v], 1), k, idx=torch.cat([bi, i], 1).contiguous())
    return bv, bi


def shard_rank(queries: torch.Tensor, shard: CatalogShard, s_label: torch.Tensor, temp: float, k: int = 50,
               q_rnorm: Optional[torch.Tensor] = None, sample: int = TOPK_SAMPLE, cap: int = TOPK_CAP,
               max_val: float = MAX_VAL):
    """One shard's part of the ranking (rf_retrieval.hip): per query the strict rank count
    #{s > s_label}, #{s > -max_val} and sum exp(s - 1/temp) over the shard, and (k > 0) the shard's
    top-k (scores descending, ties by lower item id; global ids). The scores are produced tile by
    tile and consumed in the kernel's epilogue; only a (B, sample) seed block is ever written."""
    _check_topk_args(k, sample, cap)
    q = _check_q(queries, shard)
    qn = ops.row_inv_norm(q) if q_rnorm is None else q_rnorm
    lib = _lib.load()
    B, N = q.shape[0], shard.n
    inv_t = 1.0 / temp
    dev = q.device
    s0 = min(N, sample) if k > 0 else 0
    # the dense seed: blocks of `sample` columns, their top-k merged block by block. After a seed of n_s
    # columns a row expects k * 256 / n_s candidates per 256-column tile, and the kernel stages at most
    # TILE_CAND_CAP (RK_TCAP) per (row, tile) before the row overflows into the dense re-rank: the seed is
    # sized to keep that expectation at a quarter of the cap (one block up to k = 64; 4 blocks at k = 256)
    need = 256 * k * 4 // TILE_CAND_CAP  # columns for k * 256 / n_s <= TILE_CAND_CAP / 4
    seed_n = min(N, max(s0, -(-need // sample) * sample)) if k > 0 else 0
    blocks = [(o, min(sample, seed_n - o)) for o in range(0, seed_n, sample)]
    # column chunks after the seed: each (grow - 1) times everything before it. A row expects about
    # k * (grow - 1) candidates per chunk, so the factor is capped to keep that within half the list
    # (cap): at k = 256 a growth of 8 would overflow nearly every row into the exact re-rank
    plan, off = [], seed_n
    grow = growth_for(k, cap)
    while k > 0 and off < N:
        plan.append((off, min(N - off, max(off * (grow - 1), sample))))
        off += plan[-1][1]
    nt0 = sum(lib.rf_score_rank_tiles(n) for _, n in blocks) if k > 0 else lib.rf_score_rank_tiles(N)
    ntiles = nt0 + sum(lib.rf_score_rank_tiles(n) for _, n in plan)
    part_cnt = torch.empty(ntiles, B, dtype=torch.int32, device=dev)
    part_sexp = torch.empty(ntiles, B, dtype=torch.float32, device=dev)
    topv = topi = None
    n_over = 0
    if k > 0:
        dense = torch.empty(B, (s0 + 255) // 256 * 256, dtype=torch.float32, device=dev)  # whole 256-col tiles
        tb = 0
        for o, n in blocks:
            _score_rank(q, qn, shard, s_label, inv_t, 0, o, n, part_cnt, part_sexp, tb, dense=dense, max_val=max_val)
            if topv is None:
                topv, topi = _topk_dense(dense[:, :n], k, idx_base=shard.base + o)
            elif n >= k:
                v, i = _topk_dense(dense[:, :n], k, idx_base=shard.base + o)
                topv, topi = _topk_dense(torch.cat([topv, v], 1), k, idx=torch.cat([topi, i], 1).contiguous())
            else:  # a last block narrower than k
                ids = (torch.arange(n, dtype=torch.int32, device=dev) + (shard.base + o)).expand(B, n)
                topv, topi = _topk_dense(torch.cat([topv, dense[:, :n]], 1), k,
                                         idx=torch.cat([topi, ids], 1).contiguous())
            tb += lib.rf_score_rank_tiles(n)
        del dense
        # the rest in chunks that double with the items already seen: the running k-th score is a
        # lower bound of the final one, so only s >= it can enter the top-k (about k per row per
        # chunk); each chunk's candidates are merged before the next chunk's threshold is read.
        # Rows whose candidate lists overflow keep their list (still a lower bound) and are re-ranked
        # exactly at the end.
        tn = nt0
        cval = torch.empty(B, cap, dtype=torch.float32, device=dev)
        cidx = torch.empty(B, cap, dtype=torch.int32, device=dev)
        rcnt = torch.empty(B, dtype=torch.int32, device=dev)
        over = torch.zeros(B, dtype=torch.int32, device=dev)
        for off, n in plan:
            rcnt.zero_()
            tau = topv[:, k - 1].contiguous()
            _score_rank(q, qn, shard, s_label, inv_t, 1, off, n, part_cnt, part_sexp, tn, tau=tau,
                        cand=(cval, cidx, rcnt), max_val=max_val)
            mv = torch.empty(B, k, dtype=torch.float32, device=dev)
            mi = torch.empty(B, k, dtype=torch.int32, device=dev)
            _lib.check(lib.rf_topk_merge(B, k, topv.data_ptr(), topi.data_ptr(), cval.data_ptr(), cidx.data_ptr(),
                                         rcnt.data_ptr(), cap, k, mv.data_ptr(), mi.data_ptr(), over.data_ptr(),
                                         ops._stream(q)), "rf_topk_merge")
            topv, topi = mv, mi
            tn += lib.rf_score_rank_tiles(n)
        # the per-row counts are complete: reduce them before the host reads the overflow flags, so the
        # GPU has that work queued while the host waits (nothing is left to launch after the read)
        counts = _rank_reduce(lib, B, ntiles, part_cnt, part_sexp, dev, q)
        if plan:
            rows = torch.nonzero(over).flatten()
            n_over = rows.numel()
            if rows.numel():  # many near-equal scores overflowed the lists: exact dense re-rank
                empty_v = torch.full((rows.numel(), k), float("-inf"), device=dev)
                empty_i = torch.full((rows.numel(), k), -1, dtype=torch.int32, device=dev)
                fv, fi = _dense_topk_rows(q.index_select(0, rows).contiguous(), qn.index_select(0, rows).contiguous(),
                                          shard, s_label.index_select(0, rows).contiguous(), inv_t, k, 0, N,
                                          empty_v, empty_i)
                topv = topv.index_copy(0, rows, fv)
                topi = topi.index_copy(0, rows, fi)
    else:
        _score_rank(q, qn, shard, s_label, inv_t, 2, 0, N, part_cnt, part_sexp, 0, max_val=max_val)
        counts = _rank_reduce(lib, B, ntiles, part_cnt, part_sexp, dev, q)
    gt, valid, sexp = counts
    # overflow: rows whose candidate lists overflowed and were re-ranked densely (a count of slow rows,
    # not an error: the result is exact either way)
    return {"gt": gt, "valid": valid, "sexp": sexp, "topv": topv, "topi": topi, "shift": inv_t,
            "overflow": n_over}


def _rank_reduce(lib, B: int, ntiles: int, part_cnt, part_sexp, dev, q):
    """rf_rank_reduce: the per-tile partials summed per row in tile order -> (gt, valid, sexp)."""
    gt = torch.empty(B, dtype=torch.int32, device=dev)
    valid = torch.empty(B, dtype=torch.int32, device=dev)
    sexp = torch.empty(B, dtype=torch.float32, device=dev)
    _lib.check(lib.rf_rank_reduce(B, ntiles, part_cnt.data_ptr(), part_sexp.data_ptr(), gt.data_ptr(),
                                  valid.data_ptr(), sexp.data_ptr(), ops._stream(q)), "rf_rank_reduce")
    return gt, valid, sexp


def merge_topk(vals: torch.Tensor, ids: torch.Tensor, k: int):
    """Top-k of each row of (B, M) candidate lists (e.g. the shards' top-k side by side): scores
    descending, ties by lower id — the order rf_topk_* produce. Plain torch sorts (tiny inputs)."""
    o = torch.argsort(ids, dim=1, stable=True)
    v = torch.gather(vals, 1, o)
    i = torch.gather(ids, 1, o)
    v, o2 = torch.sort(v, dim=1, descending=True, stable=True)
    return v[:, :k], torch.gather(i, 1, o2)[:, :k]


def combine_shards(parts, k: int, group=None):
    """Combine shard results across the ranks of `group` (all-reduce of the rank
    counts and exp-sum partials, all-gather of the per-shard top-k); identity for one rank."""
    import torch.distributed as dist
    gt, valid, sexp = parts["gt"], parts["valid"], parts["sexp"]
    topv, topi = parts["topv"], parts["topi"]
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        w = dist.get_world_size(group)
        for t in (gt, valid, sexp):
            dist.all_reduce(t, group=group)
        if k > 0:
            gv = [torch.empty_like(topv) for _ in range(w)]
            gi = [torch.empty_like(topi) for _ in range(w)]
            dist.all_gather(gv, topv.contiguous(), group=group)
            dist.all_gather(gi, topi.contiguous(), group=group)
            topv, topi = merge_topk(torch.cat(gv, 1), torch.cat(gi, 1), k)
    return {"gt": gt, "valid": valid, "sexp": sexp, "topv": topv, "topi": topi, "shift": parts["shift"]}


def retrieve(queries: torch.Tensor, shard: CatalogShard, labels: torch.Tensor, metrics_ks: Sequence[int], temp: float,
             k: int = 50, group=None):
    """C5 retrieval over a sharded catalog (every rank holds all queries — all-gathered CLS vectors —
    and its own CatalogShard): Ranker(metrics_ks)(Similarity(queries, catalog) / temp, labels)
    (utils.py:76-108) without the (B, N) score matrix, plus the top-k items per query over the whole
    catalog. Returns (metrics list, top-k scores (B, k), top-k item ids (B, k))."""
    import torch.distributed as dist
    _check_topk_args(k, TOPK_SAMPLE, TOPK_CAP)
    q = _check_q(queries, shard)
    qn = ops.row_inv_norm(q)
    with _rank_family(k > 0):
        sl = label_scores(q, shard, labels, temp, qn)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(sl, group=group)  # the owner's value plus zeros: exact
        part = shard_rank(q, shard, sl, temp, k, qn)
    parts = combine_shards(part, k, group)
    loss = float((torch.log(parts["sexp"]) + parts["shift"] - sl).mean())
    return _metrics(parts["gt"], parts["valid"], loss, metrics_ks), parts["topv"], parts["topi"]


def rank_catalog(queries: torch.Tensor, items: torch.Tensor, labels: torch.Tensor, metrics_ks: Sequence[int],
                 temp: float, block: int = 65536, items_rnorm: Optional[torch.Tensor] = None) -> List[float]:
    """Ranker(metrics_ks)(Similarity(queries, items) / temp, labels) without the (B, N) score matrix
    (finetune.py:70-92 over a whole catalog). Returns the Ranker's list
    [NDCG@k, HR@k ..., MRR, AUC, loss].

    bf16 / fp16 queries and items of one dtype: one fused score + rank kernel pass (rf_score_rank,
    counts only) after the label scores (rf_label_scores, bit-identical to the kernel's own value
    for that column, so the strict ranks match the full-matrix Ranker); the kernel tiles the
    catalog itself. fp32 (or mixed-dtype, computed in fp32) inputs: the exact-fp32 EPI_COS GEMM over
    column blocks of `block` items, the label scores taken from the same blocks, the counts and the
    exp-sum of the cross entropy accumulated per block by rf_rank_accum."""
    if not (queries.is_cuda and items.is_cuda):
        raise _lib.RecformerHipError("rank_catalog needs ROCm device tensors (no CPU fallback)")
    if queries.dtype == items.dtype and queries.dtype in (torch.bfloat16, torch.float16):
        shard = CatalogShard(items, 0, items_rnorm)
        q = _check_q(queries, shard)
        qn = ops.row_inv_norm(q)
        with _rank_family(False):
            sl = label_scores(q, shard, labels, temp, qn)
            parts = shard_rank(q, shard, sl, temp, 0, qn)
        loss = float((torch.log(parts["sexp"]) + parts["shift"] - sl).mean())
        return _metrics(parts["gt"], parts["valid"], loss, metrics_ks)
    return _rank_catalog_blocks(queries.float().contiguous(), items.float().contiguous(), labels, metrics_ks, temp,
                                max(int(block), 1), items_rnorm)


def _rank_catalog_blocks(q: torch.Tensor, items: torch.Tensor, labels: torch.Tensor, metrics_ks: Sequence[int],
                         temp: float, block: int, items_rnorm: Optional[torch.Tensor]) -> List[float]:
    lib = _lib.load()
    B, N = q.shape[0], items.shape[0]
    dev = q.device
    inv_t = 1.0 / temp
    lab = labels.reshape(-1).to(torch.int64)
    qn = ops.row_inv_norm(q)
    rn = ops.row_inv_norm(items) if items_rnorm is None else items_rnorm.float().contiguous()
    blocks = [(c, min(block, N - c)) for c in range(0, N, block)]
    rows = torch.arange(B, device=dev)

    def scores(c, n):
        return ops.cos_scores(q, items[c:c + n], inv_t, z_rnorm=qn, items_rnorm=rn[c:c + n])

    # the label scores from the same blocks the counts see (strict ranks need the identical value)
    sl = torch.zeros(B, dtype=torch.float32, device=dev)
    cached = None
    for c, n in blocks:
        s = scores(c, n)
        inb = (lab >= c) & (lab < c + n)
        sl = torch.where(inb, s[rows, (lab - c).clamp(0, n - 1)], sl)
        if len(blocks) == 1:
            cached = s
    gt = torch.zeros(B, dtype=torch.int32, device=dev)
    valid = torch.zeros(B, dtype=torch.int32, device=dev)
    sexp = torch.zeros(B, dtype=torch.float32, device=dev)
    sl = sl.contiguous()
    for c, n in blocks:
        s = cached if cached is not None else scores(c, n)
        _lib.check(lib.rf_rank_accum(B, n, s.data_ptr(), s.stride(0), sl.data_ptr(), float(MAX_VAL), float(inv_t),
                                     gt.data_ptr(), valid.data_ptr(), sexp.data_ptr(), ops._stream(s)),
                   "rf_rank_accum")
    loss = float((torch.log(sexp) + inv_t - sl).mean())
    return _metrics(gt, valid, loss, metrics_ks)
