"""Ranker — drop-in for the reference's evaluation metrics (utils.py:76-108; callers
finetune.py:70-92, evaluate_seq.py:35-52).

forward(scores, labels) -> [NDCG@k, Recall@k for k in ks] + [MRR, AUC, loss], Python floats as
the reference returns them. The per-row counts (rank = #{n: s_n > s_label}, strict;
valid_length = #{n: s_n > -MAX_VAL}) come from rf_rank_accum and the cross entropy from
rf_cross_entropy_fwd; only the final means are torch reductions. Works on score blocks of any
width (the counts accumulate), so a catalog can also be ranked block by block.
"""
from __future__ import annotations

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
        rank = gt.float()
        res = []
        for k in self.ks:
            indicator = (rank < k).float()
            res.append(((1 / torch.log2(rank + 2)) * indicator).mean().item())  # ndcg@k
            res.append(indicator.mean().item())  # hr@k
        res.append((1 / (rank + 1)).mean().item())  # MRR
        res.append((1 - (rank / valid.float())).mean().item())  # AUC
        return res + [loss]


def rank_catalog(queries: torch.Tensor, items: torch.Tensor, labels: torch.Tensor, metrics_ks: Sequence[int],
                 temp: float, block: int = 65536, items_rnorm: Optional[torch.Tensor] = None) -> List[float]:
    """Ranker(metrics_ks)(Similarity(queries, items) / temp, labels) without the (B, N) score matrix
    (finetune.py:70-92 over a whole catalog): the cosine scores are produced
    `block` columns at a time into one reused buffer by the EPI_COS GEMM and folded into the
    per-row counts (rf_rank_accum: strict rank, valid length) and the cross entropy's sum of
    exp(s - 1/temp) (|s| <= 1/temp, so no row max is needed). The label scores are the same
    kernel's values (the diagonal of the queries x label-items product), so the strict counts
    match the full-matrix Ranker. Returns the Ranker's list [NDCG@k, HR@k ..., MRR, AUC, loss]."""
    lib = _lib.load()
    if not (queries.is_cuda and items.is_cuda):
        raise _lib.RecformerHipError("rank_catalog needs ROCm device tensors (no CPU fallback)")
    B, N = queries.shape[0], items.shape[0]
    inv_t = 1.0 / temp
    shift = inv_t  # |cos| <= 1
    qn = ops.row_inv_norm(queries)
    rn = ops.row_inv_norm(items) if items_rnorm is None else items_rnorm
    lab = labels.reshape(-1).long()
    s_label = ops.cos_scores(queries, items.index_select(0, lab).contiguous(), inv_t, z_rnorm=qn,
                             items_rnorm=rn.index_select(0, lab).contiguous()).diagonal().contiguous()
    gt = torch.zeros(B, dtype=torch.int32, device=queries.device)
    valid = torch.zeros_like(gt)
    sexp = torch.zeros(B, dtype=torch.float32, device=queries.device)
    blk = min(block, N)
    buf = torch.empty(B, (blk + 7) // 8 * 8, dtype=torch.float32, device=queries.device)
    stream = torch.cuda.current_stream(queries.device).cuda_stream
    for off in range(0, N, blk):
        n = min(blk, N - off)
        sc = ops.cos_scores(queries, items[off:off + n], inv_t, z_rnorm=qn, items_rnorm=rn[off:off + n],
                            out=buf[:, :n])
        _lib.check(lib.rf_rank_accum(B, n, sc.data_ptr(), sc.stride(0), s_label.data_ptr(), float(MAX_VAL),
                                     float(shift), gt.data_ptr(), valid.data_ptr(), sexp.data_ptr(), stream),
                   "rf_rank_accum")
    loss = float((torch.log(sexp) + shift - s_label).mean())
    rank = gt.float()
    res = []
    for k in metrics_ks:
        indicator = (rank < k).float()
        res.append(((1 / torch.log2(rank + 2)) * indicator).mean().item())  # ndcg@k
        res.append(indicator.mean().item())  # hr@k
    res.append((1 / (rank + 1)).mean().item())  # MRR
    res.append((1 - (rank / valid.float())).mean().item())  # AUC
    return res + [loss]
