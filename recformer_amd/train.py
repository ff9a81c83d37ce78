"""Training path (autograd) for the Recformer encoder (SURVEY.md §8a A9/A10 with gradients).

Forward runs the same HIP kernels as inference; each is wrapped in a torch.autograd.Function
whose backward is written out explicitly:

  _Gemm        C = A.W^T + b (optional q-scale on the first columns)      TF:504-514, 1064-1130
               backward: dA = dC.W (rf_gemm against a transposed weight copy), dW = dC^T.A
               (rf_weight_grad: MFMA, transposed LDS reads, deterministic split reduction),
               db = colsum(dC)
  _LayerNorm   y = LN(x) from the HIP kernel (row stats saved)             TF:1071, 1130
               backward: the standard closed form in fp32, one HIP pass (rf_layernorm_bwd:
               dx per row, dgamma / dbeta as deterministic column sums)
  _EmbedLN     LN(Ew[id] + Ep[pos] + Et[tt] + Ei[ip])                       models.py:108-138
               backward: rf_embed_ln_bwd (LN backward, the pre-LN sum regathered) and, per table,
               rf_segment_rows_sum over the stably sorted token indices — deterministic, no
               atomics (no gradient at padding_idx rows of the word / position tables, as
               nn.Embedding)
  _Attention   sliding-window local + global attention (band kernel + global fold)
               TF:482-1057; backward (bf16): the local branch on the HIP backward kernels
               (rf_attn_bwd.hip; global-key columns reduced per sequence here), the global
               rows in closed form (_global_bwd); fp32 mode: an fp32 recompute of both.

Mixed precision follows the reference's autocast run (finetune.py:106-110): GEMM operands in
bf16, LayerNorm outputs / residual stream / losses in fp32, parameters fp32 (the bf16 weight
copies are autograd-tracked casts, so gradients reach the fp32 masters).

Dropout: hidden dropout (embeddings, attention output, FFN output; TF:1069, 1128, models.py:137)
is applied with torch's RNG, except in the bf16 path's fused dropout + residual + LayerNorm
(_DropAddLN), whose keep mask is a counter hash of a seed drawn from torch's RNG.
Attention-probability dropout (TF:585-586, 1036-1037): the band kernels apply and regenerate a
counter-hash mask per (sequence, head, query, key) (rf_band_attn_fwd_drop / _bwd_drop); the
global query rows use the same hash as torch ops (recformer_amd/dropout.py). The masks cannot
equal torch's RNG draws, so dropout-on runs match the reference in distribution, not bitwise.
"""
from __future__ import annotations

import contextlib
import math
import weakref
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import dropout, ops

__all__ = ["encode_train", "cos_scores_train", "cross_entropy_train"]

# the global rows' backward in closed form (_global_bwd); False: autograd over _global_torch
GLOBAL_BWD_CLOSED_FORM = True
# the closed form with its products over h merged into three batched GEMMs (False: six)
GLOBAL_BWD_MERGED = True
# bf16 training: the global branch's dh straight from a bf16-operand product (no fp32 (B*Lp, D) pass)
GLOBAL_BWD_DH16 = True
# the global-key / -value row gradients as one block-diagonal batched product per sequence (no copy)
GLOBAL_KV_BLOCKDIAG = True
# weight gradients of the layer GEMMs as a split-K batched GEMM (_weight_grad)
DW_SPLIT_K = True
# embedding + LayerNorm backward on the HIP kernels (deterministic table gradients, no index_add_)
EMBED_BWD_HIP = True
# global rows' backward on rf_global_fold_bwd_full (one pass over h from the forward's fold workspace,
# the per-head products with the key/value weights and the weight gradients inside)
GLOBAL_BWD_HIP = True
# the bias gradients of the attention-output and FFN2 Linears from the LayerNorm backward pass that
# writes their dC (rf_drop_add_ln_bwd_tb) instead of a separate column-sum pass over dC
LN_BIAS_GRAD = True
# packed bf16 / fp16 training with the HIP global backward: the query_global projection of the global
# rows runs inside _Attention, its backward on rf_global_query_bwd (dWqg, dbqg, and the rows' input
# gradient added into the branch's dh in place: no gather backward, zero fill or extra dh sum)
GLOBAL_QG_INSIDE = True
# the global-key / -value rows' gradients of the local branch on rf_global_kv_grad (one launch,
# added in place into dk / dv) instead of two batched products, their copies and a scatter
GLOBAL_KV_HIP = True
# weight gradients on the HIP kernel (rf_weight_grad: MFMA, transposed LDS reads, fixed-order split
# reduction) instead of hipBLASLt
DW_HIP = True
# bf16: FFN1 + GELU as one GEMM that also writes the pre-activation (_GemmGelu). Off: measured
# neutral at C3 (25.8 vs 26.4 ms median, alternating A/B) — the GELU moves into the GEMM's
# unhidden epilogue and the pre-activation is still written
FUSED_GELU = False
# 16-bit: the whole feed-forward block as one autograd node (_FFN): GELU in the FFN1 epilogue, its
# backward in the epilogue of the dA GEMM of FFN2, both dA GEMMs on rf_gemm
FFN_FUSED = True
# 16-bit: dA = dC.W of the other Linears (qkv, query_global, out-proj) on rf_gemm against a
# transposed weight copy instead of hipBLASLt
DA_RF_GEMM = True
# below this many rows (the global query rows' Linear: B*G rows) the backward's dA / dW are single
# library GEMMs: the 256 x 256-tile kernels would run one mostly empty K-step per tile
SMALL_M = 512


# ------------------------------------------------------------------------------------------
def _mm_f32(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """x @ y (2-D or batched 3-D) with an fp32 result: hipBLASLt's fp32 output from bf16 operands
    on the GPU (no bf16 rounding of the product), a cast elsewhere."""
    f = torch.bmm if x.dim() == 3 else torch.mm
    if x.is_cuda and x.dtype != torch.float32:
        return f(x, y, out_dtype=torch.float32)
    return f(x, y).float()


# weight gradients on a side stream beside the main stream's dA GEMM: the dA GEMMs of the N = 768
# Linears at the reference's finetune batch (16 x 1024 tokens) have 192 tiles of 256^2 for 256 CUs, so
# a quarter of the chip would idle; the independent dW = dC^T A work fills it (forked and joined with
# stream events — graph-capturable)
DW_SIDE_STREAM = True
# the global rows' attention backward (rf_global_fold_bwd_full + rf_global_query_bwd: launches of a few
# hundred workgroups) on that side stream beside the local branch's backward (_Attention.backward)
GLOBAL_BWD_SIDE = True
# the training forward's global-row fold (query projection, u, the pass over h) on that side stream beside
# the band attention, its merge + output after it (_Attention.forward, rf_global_attn_fold_fwd_stage)
FOLD_SIDE_TRAIN = True
# the attention's gradient of a layer's input added inside the q|k|v projection's dA GEMM (_GradMailbox)
# instead of autograd's separate bf16 sum: -0.4% per captured C3 step (16.55 vs 16.62 ms, gpurun_out/r04r),
# The round-4 suite fault with it on (an illegal address in the first training test after the graph tests,
# gpurun_out/r04v) was _zero_bias caching a zero vector allocated during a graph capture: it lived in that
# graph's private pool, which was freed with the graph, and every later uncaptured mailbox GEMM read it
# (fixed in _zero_bias: nothing made during a capture is cached)
GRAD_MAILBOX = True
# the bias gradients' column sums on the weight-gradient side stream too: measured slower (captured C3
# 16.48 vs 16.38 ms in one process, gpurun_out/r04s: that stream is the step's critical path), so off;
# for the q|k|v projection's sums alone also slower (15.87 vs 15.81 ms, gpurun_out/r05k)
BIAS_GRAD_SIDE = False
_SIDE_STREAMS = {}


def _dw_async(fn, ref: torch.Tensor):
    """Run fn() (weight-gradient work reading tensors the main stream produced) on a side stream
    that first waits for the main stream; returns join(), which makes the main stream wait for the
    side stream and returns fn's result (recorded on the main stream for the caching allocator)."""
    if not (DW_SIDE_STREAM and ref.is_cuda):
        r = fn()
        return lambda: r
    main = torch.cuda.current_stream(ref.device)
    side = _SIDE_STREAMS.get(ref.device)
    if side is None:
        side = _SIDE_STREAMS[ref.device] = torch.cuda.Stream(ref.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        r = fn()

    def record(x):
        if isinstance(x, torch.Tensor):
            x.record_stream(main)
        elif isinstance(x, (list, tuple)):
            for t in x:
                record(t)
        elif isinstance(x, dict):
            for t in x.values():
                record(t)

    def join():
        main.wait_stream(side)
        record(r)
        return r
    return join


# weight gradients accumulated into the masters' .grad on the side stream, with ONE join at the end of the
# backward pass (an autograd engine callback) instead of one per Linear: the main stream no longer waits
# for each layer's dW before going on (the weight-gradient stream was the step's critical path).
# Only for leaf masters without post-accumulate hooks (a DP GradBucketer's hooks, or non-leaf masters such
# as pretraining's shared casts, keep the per-Linear join and autograd's accumulation). Off by default: the
# Linears then return no gradient for their weights to autograd, so torch.autograd.grad(loss, params) would
# see none; the training drivers that own the step turn it on around their backward
# (deferred_weight_grads(): graphs.CapturedTrainStep, tools/train_bench.py).
DEFER_DW = False
_DEFER = {"queued": False}


@contextlib.contextmanager
def deferred_weight_grads(on: bool = True):
    """Within: loss.backward() accumulates the Linear weight gradients into .grad on the side stream with
    one join when the backward pass ends (DEFER_DW)."""
    global DEFER_DW
    old, DEFER_DW = DEFER_DW, on
    try:
        yield
    finally:
        DEFER_DW = old


def _defer_ok(masters, need) -> bool:
    if not (DEFER_DW and DW_SIDE_STREAM):
        return False
    for m, n in zip(masters, need):
        if n and (m is None or not m.is_leaf or not m.is_cuda or getattr(m, "_post_accumulate_grad_hooks", None)
                  or m.dtype != torch.float32):
            return False
    return True


def _accum_grad(p: torch.Tensor, g: torch.Tensor) -> None:
    """p.grad += g on the current (side) stream; the first gradient is stored as it is (AccumulateGrad's
    steal), detached from any graph."""
    if p.grad is None:
        p.grad = g.detach()
    else:
        p.grad.add_(g)


def _dw_deferred(fn, ref: torch.Tensor) -> None:
    """Run fn() (weight-gradient work that accumulates into leaf .grad tensors itself) on the side stream
    after the main stream's work so far; the main stream waits for the side stream once, when the backward
    pass ends (queued engine callback), before any optimizer or scaler reads a gradient."""
    main = torch.cuda.current_stream(ref.device)
    side = _SIDE_STREAMS.get(ref.device)
    if side is None:
        side = _SIDE_STREAMS[ref.device] = torch.cuda.Stream(ref.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in out:
        if isinstance(t, torch.Tensor):
            t.record_stream(main)
    if not _DEFER["queued"]:
        _DEFER["queued"] = True

        def join():
            _DEFER["queued"] = False
            main.wait_stream(side)
        torch.autograd.Variable._execution_engine.queue_callback(join)


def _weight_grad(dc: torch.Tensor, a: torch.Tensor, scale=(0, 1.0)) -> torch.Tensor:
    """dW = dC^T A (N, K) in fp32 (the master weight's dtype), reduced over the M = B*Lp token
    rows, its first scale[0] rows multiplied by scale[1] (a column-scaled Linear: the query's 1/8).
    The layer weights are small (N*K <= 3072*768: at most 36 tiles of 256^2) against a long
    reduction, so one GEMM leaves most of the chip idle; with DW_SPLIT_K the rows are split into
    S chunks computed as one batched GEMM (S times the tiles) and the S fp32 partials summed."""
    sc, s = scale
    if sc > 0 and s != 1.0 and not _dw_hip_ok(dc, a):
        dw = _weight_grad(dc, a)
        dw[:sc].mul_(s)
        return dw
    M, N = dc.shape
    K = a.shape[1]
    if _dw_hip_ok(dc, a):
        # any M, including a few rows (the global query rows, the CLS-only last layer): the buffer
        # resources read rows past M as zeros — no library GEMM (and no library workspace on the
        # weight-gradient side stream, which a captured graph would own)
        return ops.weight_grad(dc, a, scale_rows=sc, row_scale=s)
    if M < SMALL_M and dc.is_cuda and dc.dtype != torch.float32:
        return _mm_f32(dc.t(), a)
    S = 1
    if DW_SPLIT_K and M >= 8192 and N * K <= 4 * 1024 * 1024:
        S = 8
        while S > 1 and (M % S or M // S < 2048):
            S //= 2
    if S == 1:
        return _mm_f32(dc.t(), a)
    part = _mm_f32(dc.reshape(S, M // S, N).transpose(1, 2), a.reshape(S, M // S, K))  # (S, N, K)
    return part.sum(0)


def _dw_hip_ok(dc: torch.Tensor, a: torch.Tensor) -> bool:
    N, K = dc.shape[1], a.shape[1]
    return (DW_HIP and dc.is_cuda and dc.dtype in (torch.bfloat16, torch.float16) and a.dtype == dc.dtype
            and N % 16 == 0 and K % 16 == 0 and dc.stride(1) == 1 and a.stride(1) == 1
            and dc.stride(0) % 8 == 0 and a.stride(0) % 8 == 0
            and dc.data_ptr() % 16 == 0 and a.data_ptr() % 16 == 0)


class _Gemm(torch.autograd.Function):
    """C = A.W^T + b on rf_gemm with W's compute-dtype copy w16 (not tracked); the gradient goes
    to the master W (fp32 under autocast) directly, as fp32 dW — no cast node per weight."""

    @staticmethod
    def forward(ctx, a, w, w16, b, scale_cols: int, col_scale: float):
        ctx.save_for_backward(a, w16)
        ctx.sc = (scale_cols, col_scale)
        ctx.wdt = w.dtype
        return ops.gemm(a.contiguous(), w16, b, ops.RF_EPI_BIAS, scale_cols=scale_cols, col_scale=col_scale)

    @staticmethod
    def backward(ctx, dc):
        a, w = ctx.saved_tensors
        sc, s = ctx.sc
        dc = dc.to(a.dtype)
        scaled = sc > 0 and s != 1.0
        # the column scale of the first sc outputs goes on the small operands (W rows, dW rows,
        # db) instead of a scaled copy of dC
        wa = w
        if scaled and ctx.needs_input_grad[0]:
            wa = w.clone()
            wa[:sc] *= s
        da = None
        if ctx.needs_input_grad[0]:
            if DA_RF_GEMM and dc.dtype != torch.float32 and dc.shape[1] % 64 == 0 and wa.shape[1] % 8 == 0:
                da = ops.gemm(dc.contiguous(), wa.t().contiguous(), None, ops.RF_EPI_NONE)  # rf_gemm, W^T copy
            else:
                da = dc @ wa
        # the dW rows and db entries of the scaled outputs scaled inside the reduction kernels
        dw = _weight_grad(dc, a, (sc, s)).to(ctx.wdt) if ctx.needs_input_grad[1] else None
        db = _bias_grad(dc, (sc, s)) if ctx.needs_input_grad[3] else None  # deterministic HIP column sums
        return da, dw, None, db, None, None


def _bias_grad(dc, scale=(0, 1.0)):
    """Column sums of dC (a Linear's bias gradient), the first scale[0] multiplied by scale[1]: the ones
    the LayerNorm backward computed with dC (_DropAddLN, LN_BIAS_GRAD) when dc is that very tensor,
    else rf_colsum."""
    sc, s = scale
    cs = getattr(dc, "_rf_colsum", None)
    if cs is None:
        return ops.colsum(dc, sc, s)
    if sc > 0 and s != 1.0:
        cs = cs.clone()
        cs[:sc].mul_(s)
    return cs


class _GradMailbox:
    """One layer's hand-off of h's gradient from the attention's backward to the q|k|v projection's
    backward: h (the LayerNorm output) feeds both, so autograd would add their two bf16 gradients in a
    separate pass over (M, d); instead _Attention.backward leaves its part here and _GemmP.backward (which
    runs after it: it needs the attention's dq|dk|dv) adds it in the dA GEMM's epilogue (EPI_BIAS_RESID
    with a zero bias; one rounding to bf16 instead of two)."""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None


_ZERO_BIAS = {}


def _zero_bias(n: int, device) -> torch.Tensor:
    """A zero bias vector for the residual-form GEMM. Cached only when made outside a graph capture: a
    tensor allocated while capturing lives in that graph's private pool and is freed with the graph,
    so a cached one would dangle for every later step."""
    t = _ZERO_BIAS.get((n, device))
    if t is None:
        t = torch.zeros(n, dtype=torch.float32, device=device)
        if not torch.cuda.is_current_stream_capturing():
            _ZERO_BIAS[(n, device)] = t
    return t


class _GemmP(torch.autograd.Function):
    """_Gemm over packed weights (ops.WeightPack, one rf_pack_weights launch per forward): the forward
    reads the compute-dtype copy w16, the backward's dA = dC.W the packed transposed copy w16t (its
    first scale_cols rows already multiplied by col_scale), and dW = dC^T.A is split by rows over the
    masters — the fused q|k|v weight's three nn.Linear weights get their gradients as row blocks of
    one rf_weight_grad result, with no concatenation in the forward and no split copy."""

    @staticmethod
    def forward(ctx, a, b, w16, w16t, scale_cols: int, col_scale: float, mb, *masters):
        ctx.save_for_backward(a, w16t)
        ctx.mb = mb  # a _GradMailbox (or None): another consumer's gradient of a, added into dA
        ctx.sc = (scale_cols, col_scale)
        ctx.rows = [m.shape[0] for m in masters]
        ctx.wdt = masters[0].dtype
        ctx.masters = masters
        return ops.gemm(a.contiguous(), w16, b, ops.RF_EPI_BIAS, scale_cols=scale_cols, col_scale=col_scale)

    @staticmethod
    def backward(ctx, dc):
        a, wt = ctx.saved_tensors
        sc, s = ctx.sc
        dc = dc.to(a.dtype).contiguous()
        scaled = sc > 0 and s != 1.0
        da = None
        # the dW rows and db entries of the scaled outputs scaled inside the reduction kernels
        scl = (sc, s) if scaled else (0, 1.0)
        side_b = BIAS_GRAD_SIDE and ctx.needs_input_grad[1] and any(ctx.needs_input_grad[7:])
        need_w = ctx.needs_input_grad[7:]
        join = None
        if any(need_w) and not side_b and dc.is_cuda and _defer_ok(ctx.masters, need_w):
            rows, masters = ctx.rows, ctx.masters

            def side_work():
                dw = _weight_grad(dc, a, scl).to(ctx.wdt)
                r0 = 0
                for m, n, nd in zip(masters, rows, need_w):
                    if nd:
                        _accum_grad(m, dw[r0:r0 + n])
                    r0 += n
                return (dw,)
            _dw_deferred(side_work, dc)
            need_w = (False,) * len(need_w)  # accumulated on the side stream, returned as None
        elif any(need_w):
            join = _dw_async(lambda: (_weight_grad(dc, a, scl).to(ctx.wdt), _bias_grad(dc, scl) if side_b else None),
                             dc)
        if ctx.needs_input_grad[0]:
            other = ctx.mb.g if ctx.mb is not None else None
            if other is not None:  # dA + the attention's gradient of the same input, in the epilogue
                ctx.mb.g = None
                da = ops.gemm(dc, wt, _zero_bias(wt.shape[0], dc.device), ops.RF_EPI_BIAS_RESID, resid=other)
            else:
                da = ops.gemm(dc, wt, None, ops.RF_EPI_NONE)  # any M (a few rows: the small-tile kernel)
        db = _bias_grad(dc, scl) if ctx.needs_input_grad[1] and not side_b else None
        dw = None
        if join is not None:
            dw, dbs = join()
            db = dbs if side_b else db
        dws = [None] * len(ctx.rows)
        if dw is not None:
            r0 = 0
            for i, n in enumerate(ctx.rows):
                dws[i] = dw[r0:r0 + n] if need_w[i] else None
                r0 += n
        return (da, db, None, None, None, None, None, *dws)


class _GemmGelu(torch.autograd.Function):
    """u = gelu(A.W^T + b) (TF:1107-1116) in one rf_gemm (EPI_BIAS_GELU_AUX), which also writes
    the bf16 pre-activation z the GELU backward needs (no separate GELU pass over z)."""

    @staticmethod
    def forward(ctx, a, w, w16, b):
        a = a.contiguous()
        z = torch.empty(a.shape[0], w16.shape[0], dtype=a.dtype, device=a.device)
        u = ops.gemm(a, w16, b, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
        ctx.save_for_backward(a, w16, z)
        ctx.wdt = w.dtype
        return u

    @staticmethod
    def backward(ctx, du):
        a, w, z = ctx.saved_tensors
        dz = torch.ops.aten.gelu_backward(du.to(z.dtype), z)  # exact-erf GELU', as F.gelu's backward
        da = dz @ w if ctx.needs_input_grad[0] else None
        dw = _weight_grad(dz, a).to(ctx.wdt) if ctx.needs_input_grad[1] else None
        db = ops.colsum(dz) if ctx.needs_input_grad[3] else None
        return da, dw, None, db


class _DecoderCE(torch.autograd.Function):
    """LongformerLMHead.decoder + the masked-LM CrossEntropyLoss (TF:1283-1285, models.py:499-510)
    for 16-bit compute: logits on rf_gemm in the compute dtype, the loss rows on
    rf_cross_entropy_fwd (fp32 log-sum-exp), and in the backward d(loss)/d(logits) written in the
    compute dtype by one kernel (rf_cross_entropy_bwd: softmax - one-hot, scaled on the device), so
    no fp32 log-softmax / probability matrix of (rows x vocab) is materialised; dX and dW from it
    as for every other Linear (dW in fp32 for the master weight)."""

    @staticmethod
    def forward(ctx, x, w, b, labels, ignore_index: int):
        w16 = w.detach().to(x.dtype).contiguous()
        logits = ops.gemm(x.contiguous(), w16, b.detach().float().contiguous(), ops.RF_EPI_BIAS)
        rows = ops.cross_entropy(logits, labels, ignore_index, reduction="none")
        n = (labels.reshape(-1) != ignore_index).sum().to(torch.float32)
        ctx.save_for_backward(x, w16, logits, labels, n)
        ctx.ign = ignore_index
        ctx.wdt = w.dtype
        return rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        x, w16, logits, labels, n = ctx.saved_tensors
        dlog = ops.cross_entropy_bwd(logits, labels, (g.float() / n).reshape(1), ctx.ign)
        dx = dlog @ w16 if ctx.needs_input_grad[0] else None
        dw = _weight_grad(dlog, x.contiguous()).to(ctx.wdt) if ctx.needs_input_grad[1] else None
        db = ops.colsum(dlog) if ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None


class _CosScores(torch.autograd.Function):
    """Similarity(z, items) / temp for training (models.py:358-369, used by :583-599) on HIP, in fp32
    as the reference's autocast runs cosine_similarity: forward on rf_gemm's EPI_COS (exact fp32 MFMA,
    the full catalog) or rf_cos_score_cand (sampled candidates, models.py:592-597), the backward's
    dL/dz on rf_cos_score_bwd. The item table is frozen (nn.Embedding.from_pretrained(freeze=True),
    models.py:536) and its inverse norms cached by the caller, so nothing flows to it and it is never
    re-normalised per step."""

    @staticmethod
    def forward(ctx, zf, table, t_rnorm, cand, inv_t: float):
        rz = ops.row_inv_norm(zf)
        if cand is None:
            s = ops.cos_scores(zf, table, inv_t, z_rnorm=rz, items_rnorm=t_rnorm)
        else:
            s = ops.cos_scores_cand(zf, table, cand, inv_t, z_rnorm=rz, items_rnorm=t_rnorm)
        ctx.save_for_backward(zf, rz, table, t_rnorm, s, cand if cand is not None else torch.empty(0))
        ctx.sampled = cand is not None
        ctx.inv_t = inv_t
        return s

    @staticmethod
    def backward(ctx, g):
        zf, rz, table, t_rnorm, s, cand = ctx.saved_tensors
        dz = ops.cos_scores_bwd(zf, table, g.float().contiguous(), s, ctx.inv_t, rz, t_rnorm,
                                cand if ctx.sampled else None)
        return dz, None, None, None, None


class _CrossEntropy(torch.autograd.Function):
    """torch.nn.functional.cross_entropy (mean over the non-ignored rows) of fp32 logits on
    rf_cross_entropy_fwd / rf_cross_entropy_bwd (softmax - one-hot, scaled on the device): the
    finetuning loss of models.py:589-597."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index: int = -100):
        rows = ops.cross_entropy(logits, labels, ignore_index, reduction="none")
        n = (labels.reshape(-1) != ignore_index).sum().to(torch.float32)
        ctx.save_for_backward(logits, labels, n)
        ctx.ign = ignore_index
        return rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        logits, labels, n = ctx.saved_tensors
        dlog = ops.cross_entropy_bwd(logits, labels, (g.float() / n).reshape(1), ctx.ign)
        return dlog, None, None


def cos_scores_train(z: torch.Tensor, table: torch.Tensor, t_rnorm: torch.Tensor, inv_t: float,
                     cand: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Differentiable fp32 cosine scores of z against a frozen fp32 table (inverse norms given)."""
    return _CosScores.apply(z.float().contiguous(), table, t_rnorm, cand, float(inv_t))


def cross_entropy_train(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    return _CrossEntropy.apply(logits, labels.reshape(-1).to(torch.int64).contiguous(), ignore_index)


class _LMHeadTransform(torch.autograd.Function):
    """LongformerLMHead's dense -> exact GELU -> LayerNorm (TF:1277-1282) for 16-bit compute, the
    reference's autocast semantics: dense on rf_gemm with the bias + GELU epilogue writing both
    gelu(z) and the pre-activation z in the compute dtype (EPI_BIAS_GELU_AUX), LayerNorm of that
    16-bit tensor in fp32 on rf_layernorm_fwd, its output rounded to the compute dtype (the decoder's
    operand — autocast's cast of the fp32 LayerNorm output). Backward: rf_layernorm_bwd in fp32, the
    exact-erf GELU backward in the compute dtype (as autograd of F.gelu on a 16-bit tensor), dX on
    rf_gemm (transposed weight copy), dW as every Linear's (_weight_grad, fp32), db / dgamma / dbeta
    as deterministic column sums."""

    @staticmethod
    def forward(ctx, x, w, w16, b, ln_w, ln_b, eps: float):
        x = x.contiguous()
        z = torch.empty(x.shape[0], w16.shape[0], dtype=x.dtype, device=x.device)
        u = ops.gemm(x, w16, b, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
        lw = ln_w.float().contiguous()
        y, mean, rstd = ops.layernorm(u, lw, ln_b.float().contiguous(), eps, out_dtype=x.dtype, stats=True)
        ctx.save_for_backward(x, w16, z, u, mean, rstd, lw)
        ctx.wdt = w.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w16, z, u, mean, rstd, lw = ctx.saved_tensors
        du, dlw, dlb = ops.layernorm_bwd(dy.float(), u.float(), mean, rstd, lw)
        dz = torch.ops.aten.gelu_backward(du.to(z.dtype), z).contiguous()
        dx = ops.gemm(dz, w16.t().contiguous(), None, ops.RF_EPI_NONE) if ctx.needs_input_grad[0] else None
        dw = _weight_grad(dz, x).to(ctx.wdt) if ctx.needs_input_grad[1] else None
        db = ops.colsum(dz) if ctx.needs_input_grad[3] else None
        return dx, dw, None, db, dlw, dlb, None


def lm_head_transform(x, dense_w, dense_b, ln_w, ln_b, eps: float):
    """gelu(x.W^T + b) -> LayerNorm, in x's 16-bit dtype (see _LMHeadTransform)."""
    return _LMHeadTransform.apply(x, dense_w, dense_w.detach().to(x.dtype).contiguous(), dense_b.float(), ln_w,
                                  ln_b, eps)


def decoder_ce(x, w, b, labels, ignore_index: int = -100):
    """Mean cross entropy of x.W^T + b against labels (16-bit x; see _DecoderCE)."""
    return _DecoderCE.apply(x, w, b, labels.reshape(-1), ignore_index)


class _FFN(torch.autograd.Function):
    """The feed-forward block's two Linears around the exact GELU (TF:1107-1116, 1123-1126) for
    16-bit compute, t2 = gelu(a.W1^T + b1).W2^T + b2: forward FFN1 with EPI_BIAS_GELU_AUX (GELU
    output + the pre-activation z in one GEMM), FFN2 with EPI_BIAS; backward dz = (dt2.W2) *
    gelu'(z) as ONE rf_gemm (EPI_DGELU, against a transposed copy of W2) — no du tensor and no
    separate GELU-backward pass — and da = dz.W1 on rf_gemm too (transposed copy of W1); the
    weight gradients (long token reductions) as for every Linear (_weight_grad, fp32)."""

    @staticmethod
    def forward(ctx, a, w1, w1_16, b1, w2, w2_16, b2, w1t=None, w2t=None):
        a = a.contiguous()
        z = torch.empty(a.shape[0], w1_16.shape[0], dtype=a.dtype, device=a.device)
        u = ops.gemm(a, w1_16, b1, ops.RF_EPI_BIAS_GELU_AUX, resid=z)
        t2 = ops.gemm(u, w2_16, b2, ops.RF_EPI_BIAS)
        # the transposed copies dA needs: packed ones (ops.WeightPack) when given, else made here
        ctx.save_for_backward(a, u, z, w1_16 if w1t is None else w1t, w2_16 if w2t is None else w2t)
        ctx.packed = (w1t is not None, w2t is not None)
        ctx.wdt = (w1.dtype, w2.dtype)
        ctx.masters = (w1, w2)
        return t2

    @staticmethod
    def backward(ctx, dt2):
        a, u, z, w1, w2 = ctx.saved_tensors
        w1t = w1 if ctx.packed[0] else w1.t().contiguous()
        w2t = w2 if ctx.packed[1] else w2.t().contiguous()
        dt2 = dt2.to(a.dtype).contiguous()
        dz = ops.gemm(dt2, w2t, None, ops.RF_EPI_DGELU, resid=z)
        db2 = _bias_grad(dt2) if ctx.needs_input_grad[6] else None
        # both weight gradients on the side stream, beside da = dz.W1 (N = 768: a quarter of the CUs
        # idle at 16k tokens); dw2 waits for nothing but dt2, dw1 for dz
        side_b = BIAS_GRAD_SIDE and ctx.needs_input_grad[3]
        need1, need2 = ctx.needs_input_grad[1], ctx.needs_input_grad[4]
        w1m, w2m = ctx.masters
        join = None
        if (need1 or need2) and not side_b and dz.is_cuda and _defer_ok((w1m, w2m), (need1, need2)):
            def side_work():
                dw2 = _weight_grad(dt2, u).to(ctx.wdt[1]) if need2 else None
                if need2:
                    _accum_grad(w2m, dw2)
                dw1 = _weight_grad(dz, a).to(ctx.wdt[0]) if need1 else None
                if need1:
                    _accum_grad(w1m, dw1)
                return (dw2, dw1)
            _dw_deferred(side_work, dz)
        else:
            join = _dw_async(lambda: (_weight_grad(dt2, u).to(ctx.wdt[1]) if need2 else None,
                                      _weight_grad(dz, a).to(ctx.wdt[0]) if need1 else None,
                                      ops.colsum(dz) if side_b else None), dz)
        da = ops.gemm(dz, w1t, None, ops.RF_EPI_NONE) if ctx.needs_input_grad[0] else None
        db1 = ops.colsum(dz) if ctx.needs_input_grad[3] and not side_b else None
        dw2 = dw1 = None
        if join is not None:
            dw2, dw1, db1s = join()
            db1 = db1s if side_b else db1
        return da, dw1, None, db1, dw2, None, db2, None, None


def _ln_backward(dy, x, mean, rstd, w):
    if x.dtype == torch.float32 and x.is_cuda:  # one HIP pass (rf_layernorm_bwd)
        return ops.layernorm_bwd(dy.float(), x, mean, rstd, w)
    xhat = (x.float() - mean[:, None]) * rstd[:, None]
    g = dy.float() * w[None, :]
    dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
    dw = (dy.float() * xhat).sum(0)
    db = dy.float().sum(0)
    return dx, dw, db


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps: float, out_dtype):
        y, mean, rstd = ops.layernorm(x.contiguous(), w, b, eps, out_dtype=out_dtype, stats=True)
        ctx.save_for_backward(x, mean, rstd, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, w = ctx.saved_tensors
        dx, dw, db = _ln_backward(dy, x, mean, rstd, w)
        return dx.to(x.dtype), dw, db, None, None


class _DropAddLN(torch.autograd.Function):
    """y = LN(dropout_p(t) + res) (TF:1068-1071, 1127-1130): t the bf16 dense output, res the fp32
    residual stream; one HIP pass each way (rf_drop_add_ln_fwd / _bwd), the dropout mask a
    counter hash of a seed drawn from torch's RNG. dual: also returns bf16(y), the next GEMM's
    operand, from the same pass, and the backward sums both outputs' gradients in the kernel
    (no separate cast, cast-backward and gradient add per LayerNorm)."""

    @staticmethod
    def forward(ctx, t, res, w, b, eps: float, p: float, dual: bool = False, seed: Optional[int] = None,
                mask_row_mul: int = 1):
        # mask_row_mul: rows drawn as row * mask_row_mul of the mask (the CLS-only last layer's compacted
        # CLS rows pass Lp: each gets the mask of its row b * Lp in the full layer)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        out = ops.drop_add_ln_fwd(t, res.contiguous(), w, b, eps, p, seed, want_bf16=dual, mask_row_mul=mask_row_mul)
        x, y, mean, rstd = out[:4]
        ctx.save_for_backward(x, mean, rstd, w)
        ctx.p, ctx.seed, ctx.mrow = p, seed, mask_row_mul
        ctx.tdt = t.dtype
        ctx.set_materialize_grads(False)
        return (y, out[4]) if dual else y

    @staticmethod
    def backward(ctx, dy, dy16=None):
        if dy is None and dy16 is None:
            return None, None, None, None, None, None, None, None, None
        x, mean, rstd, w = ctx.saved_tensors
        if LN_BIAS_GRAD and ctx.needs_input_grad[0]:
            # the dense branch's bias gradient (column sums of dt) from the same pass, handed to the
            # producing Linear's backward with dt (_bias_grad)
            dres, dt, dw, db, dbias = ops.drop_add_ln_bwd(dy, x, mean, rstd, w, ctx.p, ctx.seed, dy16=dy16,
                                                          dtype=ctx.tdt, want_dbias=True, mask_row_mul=ctx.mrow)
            dt._rf_colsum = dbias
        else:
            dres, dt, dw, db = ops.drop_add_ln_bwd(dy, x, mean, rstd, w, ctx.p, ctx.seed, dy16=dy16, dtype=ctx.tdt,
                                                   mask_row_mul=ctx.mrow)
        return dt, dres, dw, db, None, None, None, None, None


class _EmbedLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, pos, tt, ip, word, pe, te, ie, ln_w, ln_b, eps: float, pad_id: int):
        h, mean, rstd = None, None, None
        out = ops.embed_ln(ids, pos, tt, ip, word, pe, te, ie, ln_w, ln_b, eps, out_dtype=torch.float32)
        h = out[0] if isinstance(out, tuple) else out
        ctx.save_for_backward(ids, pos, tt, ip, word, pe, te, ie, ln_w)
        ctx.eps, ctx.pad = eps, pad_id
        return h

    @staticmethod
    def backward(ctx, dh):
        ids, pos, tt, ip, word, pe, te, ie, ln_w = ctx.saved_tensors
        if EMBED_BWD_HIP and dh.is_cuda and word.shape[1] % 4 == 0 and word.shape[1] <= 1024:
            # rf_embed_ln_bwd (LN backward with the pre-LN sum regathered) + per-table deterministic row
            # sums over the sorted token indices (rf_segment_rows_sum) — no atomics, no fp32 copy of x
            dx, dw, db = ops.embed_ln_bwd(ids, pos, tt, ip, word.contiguous(), pe.contiguous(), te.contiguous(),
                                          ie.contiguous(), ln_w, ctx.eps, dh.reshape(-1, word.shape[1]))
            grads = [ops.embedding_grad(dx, idx, table.shape[0], pad)
                     for table, idx, pad in ((word, ids, ctx.pad), (pe, pos, ctx.pad), (te, tt, None), (ie, ip, None))]
            return (None, None, None, None, *grads, dw, db, None, None)
        i, p, t, q = (x.reshape(-1).long() for x in (ids, pos, tt, ip))
        x = word[i] + pe[p] + te[t] + ie[q]  # recompute the pre-LN sum (fp32)
        mean = x.mean(-1)
        rstd = torch.rsqrt(x.var(-1, unbiased=False) + ctx.eps)
        dx, dw, db = _ln_backward(dh.reshape(x.shape), x, mean, rstd, ln_w)
        grads = []
        for table, idx, pad in ((word, i, ctx.pad), (pe, p, ctx.pad), (te, t, None), (ie, q, None)):
            g = torch.zeros_like(table).index_add_(0, idx, dx)
            if pad is not None:
                g[pad] = 0
            grads.append(g)
        return (None, None, None, None, *grads, dw, db, None, None)


# ------------------------------------------------------------------------------------------
def _local_torch(q, k, v, flags, gidx, B: int, Lp: int, H: int, half_w: int, drop=None):
    """fp32 recompute of the local branch (band keys + the local K/V rows at the global
    positions); padded query rows 0. q, k, v (B*Lp, D), q pre-scaled; flags (B, Lp)
    {0 pad, 1 local, 2 global}; gidx (B, gmax). The global query rows' values are replaced by
    the global branch in _attention_torch. drop = (p, seed): attention-probability dropout
    (TF:585-586) with the kernels' counter-hash mask (recformer_amd/dropout.py)."""
    D = q.shape[1]
    hd = D // H
    f = flags.long()
    valid = f != 0
    local = f == 1
    qh = q.float().view(B, Lp, H, hd)
    kh = k.float().view(B, Lp, H, hd)
    vh = v.float().view(B, Lp, H, hd)
    W = 2 * half_w
    nb = Lp // W
    # window keys for query block c: rows [cW - half_w, cW + W + half_w)
    kp = F.pad(kh, (0, 0, 0, 0, half_w, half_w))
    vp = F.pad(vh, (0, 0, 0, 0, half_w, half_w))
    lp = F.pad(local, (half_w, half_w))
    kw = kp.unfold(1, 2 * W, W)[:, :nb]        # (B, nb, H, hd, 2W)
    vw = vp.unfold(1, 2 * W, W)[:, :nb]
    lw = lp.unfold(1, 2 * W, W)[:, :nb]        # (B, nb, 2W)
    qb = qh.view(B, nb, W, H, hd)
    s = torch.einsum("bcihd,bchdj->bchij", qb, kw)   # (B, nb, H, W, 2W)
    ii = torch.arange(W, device=q.device)[:, None] + half_w
    jj = torch.arange(2 * W, device=q.device)[None, :]
    band = (ii - jj).abs() <= half_w
    ok = band[None, None, None] & lw[:, :, None, None, :]
    s = s.masked_fill(~ok, float("-inf"))
    gmax = gidx.shape[1]
    if gmax > 0:
        gv = gidx >= 0
        gi = gidx.clamp(min=0).long()
        kg_loc = torch.gather(kh, 1, gi[:, :, None, None].expand(B, gmax, H, hd))  # local K at globals
        vg_loc = torch.gather(vh, 1, gi[:, :, None, None].expand(B, gmax, H, hd))
        sg = torch.einsum("bcihd,bghd->bchig", qb, kg_loc)   # (B, nb, H, W, G)
        sg = sg.masked_fill(~gv[:, None, None, None, :], float("-inf"))
        s = torch.cat([s, sg], -1)
    m = s.amax(-1, keepdim=True)
    m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    p = torch.exp(s - m)
    p = p / p.sum(-1, keepdim=True).clamp_min(1e-30)
    if drop is not None and drop[0] > 0:
        dev = q.device
        bi = torch.arange(B, device=dev).view(B, 1, 1, 1, 1)
        ci = torch.arange(nb, device=dev).view(1, nb, 1, 1, 1)
        hi = torch.arange(H, device=dev).view(1, 1, H, 1, 1)
        qi = torch.arange(W, device=dev).view(1, 1, 1, W, 1)
        row = (bi * H + hi) * Lp + ci * W + qi                                  # (B, nb, H, W, 1)
        keys = ci * W - half_w + torch.arange(2 * W, device=dev).view(1, 1, 1, 1, 2 * W)
        z = dropout.attn_scale(drop[1], drop[0], row, keys, Lp)
        if gmax > 0:
            z = torch.cat([z, dropout.attn_scale(drop[1], drop[0], row, gidx.view(B, 1, 1, 1, gmax), Lp)], -1)
        p = p * z
    o = torch.einsum("bchij,bchdj->bcihd", p[..., :2 * W], vw)
    if gmax > 0:
        o = o + torch.einsum("bchig,bghd->bcihd", p[..., 2 * W:], vg_loc)
    o = o.reshape(B, Lp, H, hd) * valid[:, :, None, None]
    return o.reshape(B * Lp, D)


def _global_keep(gidx, B: int, Lp: int, H: int, p: float, seed: int):
    """Dropout scale (B, H, gmax, Lp) of the global query rows' probabilities (TF:1036-1037):
    mask row (b*H + h)*Lp + gidx[b, g], key l (the kernels' hash, recformer_amd/dropout.py)."""
    G = gidx.shape[1]
    dev = gidx.device
    row = (torch.arange(B, device=dev).view(B, 1, 1, 1) * H + torch.arange(H, device=dev).view(1, H, 1, 1)) * Lp \
        + gidx.clamp(min=0).to(torch.int64).view(B, 1, G, 1)
    return dropout.attn_scale(seed, p, row, torch.arange(Lp, device=dev).view(1, 1, 1, Lp), Lp)


def _global_torch(qg, h, wkg, bkg, wvg, bvg, flags, B: int, Lp: int, H: int, z=None):
    """Global query rows (TF:964-1057), (B*gmax, D): key_global / value_global over all tokens
    through the fold (rf_global.hip): s = (Wkg_h^T qg_h) . h_l + qg_h . bkg_h and
    out = Wvg_h (sum_l p_l h_l) + bvg_h, so no (B*Lp, D) projection is materialised and autograd
    differentiates the same algebra. z (B, H, gmax, Lp): attention-probability dropout scale
    (_global_keep); the dropped probabilities no longer sum to 1, so the value bias enters as
    bvg_h * sum_l p'_l."""
    D = h.shape[1]
    hd = D // H
    gmax = qg.shape[0] // B
    valid = flags.long() != 0
    hf = h.float().view(B, Lp, D)
    qgh = qg.float().view(B, gmax, H, hd)
    u = torch.einsum("bghd,hdk->bghk", qgh, wkg.float().view(H, hd, D))
    sgg = torch.einsum("bghk,blk->bhgl", u, hf) + torch.einsum("bghd,hd->bhg", qgh, bkg.float().view(H, hd))[..., None]
    sgg = sgg.masked_fill(~valid[:, None, None, :], float("-inf"))
    pg = torch.softmax(sgg, -1)
    if z is not None:
        pg = pg * z
    w = torch.einsum("bhgl,blk->bghk", pg, hf)
    og = torch.einsum("bghk,hdk->bghd", w, wvg.float().view(H, hd, D))
    if z is None:
        og = og + bvg.float().view(H, hd)
    else:
        og = og + pg.sum(-1).transpose(1, 2)[..., None] * bvg.float().view(H, hd)
    return og.reshape(B * gmax, D)


def _global_bwd(qg, h, wkg, wvg, flags, B: int, Lp: int, H: int, gout, z=None, bvg=None, dh_dtype=None):
    """Closed-form gradient of _global_torch (the fold algebra, TF:964-1057) for the output
    gradient gout (B*gmax, D) — batched matmuls instead of autograd over einsums (a third of the
    ops, no nested graph). Returns fp32 (dqg, dh, dwkg, dbkg, dwvg, dbvg); dbkg is exactly zero:
    the key bias adds q.bkg to every score of a row, which the softmax cancels. z (B, H, gmax, Lp):
    the forward's attention-dropout scale (then bvg, the value bias, is needed too). dh_dtype =
    torch.bfloat16: dh (the (B*Lp, D) output, rounded to bf16 by the caller anyway) is produced by a
    bf16-operand product with fp32 accumulation instead of an fp32 product and a cast (merged form)."""
    D = h.shape[1]
    hd = D // H
    G = qg.shape[0] // B
    HG = H * G
    hf = h.float().view(B, Lp, D)
    wk = wkg.float().view(H, hd, D)
    wv = wvg.float().view(H, hd, D)
    qH = qg.float().view(B * G, H, hd).transpose(0, 1)                       # (H, BG, hd)
    uH = torch.bmm(qH, wk)                                                   # (H, BG, D)
    u = uH.view(H, B, G, D).transpose(0, 1).reshape(B, HG, D)                # (B, HG, D)
    doH = gout.float().view(B * G, H, hd).transpose(0, 1)                    # (H, BG, hd)
    dwH = torch.bmm(doH, wv)                                                 # (H, BG, D)
    dw = dwH.view(H, B, G, D).transpose(0, 1).reshape(B, HG, D)
    if GLOBAL_BWD_MERGED:
        # three passes over h instead of six: [u; dw].h^T gives the scores and d/dp' together,
        # [p'; ds].h gives w and du, and dh = p'^T.dw + ds^T.u is one product with K = 2HG
        sdp = torch.bmm(torch.cat((u, dw), 1), hf.transpose(1, 2))           # (B, 2HG, Lp)
        s, dp = sdp[:, :HG], sdp[:, HG:]
    else:
        s = torch.bmm(u, hf.transpose(1, 2))                                 # (B, HG, Lp)
        dp = torch.bmm(dw, hf.transpose(1, 2))                               # (B, HG, Lp): d/dp'
    s = s.masked_fill((flags == 0).view(B, 1, Lp), float("-inf"))
    p = torch.softmax(s, -1)
    pd = p if z is None else p * z.reshape(B, HG, Lp)                        # dropped probabilities
    if z is None:
        dbvg = doH.sum(1).reshape(D)
    else:  # out += bvg * S' with S' = sum_l p'_l per (b, h, g)
        sH = pd.sum(-1).view(B, H, G).permute(1, 0, 2).reshape(H, B * G, 1)
        dbvg = (doH * sH).sum(1).reshape(D)
    if z is not None:
        dS = (doH * bvg.float().view(H, 1, hd)).sum(-1)                       # (H, BG): d/dS'
        dp = (dp + dS.view(H, B, G).permute(1, 0, 2).reshape(B, HG, 1)) * z.reshape(B, HG, Lp)
    ds = p * (dp - (p * dp).sum(-1, keepdim=True))
    if GLOBAL_BWD_MERGED:
        pds = torch.cat((pd, ds), 1)                                         # (B, 2HG, Lp)
        wdu = torch.bmm(pds, hf)                                             # (B, 2HG, D)
        w, du = wdu[:, :HG], wdu[:, HG:]
        dwu = torch.cat((dw, u), 1)                                          # (B, 2HG, D)
        if dh_dtype == torch.bfloat16:
            dh = torch.bmm(pds.transpose(1, 2).to(dh_dtype), dwu.to(dh_dtype))  # (B, Lp, D) bf16
        else:
            dh = torch.bmm(pds.transpose(1, 2), dwu)                         # (B, Lp, D)
    else:
        w = torch.bmm(pd, hf)                                                # (B, HG, D)
        dh = torch.bmm(pd.transpose(1, 2), dw).add_(torch.bmm(ds.transpose(1, 2), u))  # (B, Lp, D)
        du = torch.bmm(ds, hf)                                               # (B, HG, D)
    wH = w.reshape(B, H, G, D).transpose(0, 1).reshape(H, B * G, D)          # (H, BG, D)
    dwvg = torch.bmm(doH.transpose(1, 2), wH).reshape(D, D)                  # (H, hd, D)
    duH = du.reshape(B, H, G, D).transpose(0, 1).reshape(H, B * G, D)
    dq = torch.bmm(duH, wk.transpose(1, 2)).transpose(0, 1).reshape(B * G, D)
    dwkg = torch.bmm(qH.transpose(1, 2), duH).reshape(D, D)
    dbkg = torch.zeros(D, dtype=torch.float32, device=h.device)
    return dq, dh.view(B * Lp, D), dwkg, dbkg, dwvg, dbvg


def _fold_ws(h, B: int, Lp: int, H: int, G: int):
    """A fold workspace the training forward keeps for the HIP global backward (16-bit, D a multiple
    of 128 up to 768, at most 4 global rows per sequence, B * G <= 1024 global rows and Lp <= 4096 —
    the limits rf_global_fold_bwd_full / rf_global_query_bwd require), else None: the closed-form
    torch backward (_global_bwd) then handles the batch instead of the HIP entry points raising."""
    D = h.shape[1]
    if GLOBAL_BWD_HIP and h.is_cuda and h.dtype != torch.float32 and D % 128 == 0 and D <= 768 and G <= 4 \
            and H <= 16 and D == 64 * H and B * G <= 1024 and Lp <= 4096:
        return ops.global_fold_workspace(h, B, Lp, H, G)
    return None


def _global_bwd_hip(qg, h, wkg, wvg, bvg, flags, gidx, B: int, Lp: int, H: int, d16, ws, p_drop: float, seed: int):
    """_global_bwd on rf_global_fold_bwd_full: the global rows' whole backward from the attention output
    gradient d16 (16-bit, the global rows read at gidx) and the forward's fold workspace (one pass over
    h; the per-head products with the (d x d) weights inside); returns fp32 (dqg, dh (h's dtype), dwkg,
    dbkg, dwvg, dbvg) like _global_bwd."""
    D = h.shape[1]
    dh = torch.empty(B * Lp, D, dtype=h.dtype, device=h.device)
    dqg, dwkg, dbkg, dwvg, dbvg = ops.global_fold_bwd_full(
        h.contiguous(), flags, gidx, B, Lp, H, ws, d16, qg.contiguous(), wkg.contiguous(), wvg.contiguous(), bvg,
        p_drop, seed, dh)
    return dqg, dh, dwkg, dbkg, dwvg, dbvg


def _global_kv_grad(w, x, B: int, Lp: int, H: int):
    """Gradient of the global-key (or -value) rows, sum_i w[b,h,i,g] * x[b,i,h,:] -> (B*G, D) in x's
    dtype (bf16 operands, fp32 accumulation). w: (B, H, Lp, G) per-query score (or probability)
    gradients of the global keys; x: (B*Lp, D) rows, e.g. the q column slice of the fused qkv.
    With GLOBAL_KV_BLOCKDIAG: one batched product per sequence against x's rows in place (no
    (b, h, i, d) copy of x; x may be a strided column slice): (H*G, Lp).(Lp, D) yields every head
    pair, the diagonal head blocks are kept (12x the flops of the einsum, which are tiny, for no
    pass over x besides the product's own read)."""
    G = w.shape[-1]
    D = x.shape[1]
    if not GLOBAL_KV_BLOCKDIAG:
        return torch.einsum("bhig,bihd->bghd", w.to(x.dtype), x.reshape(B, Lp, H, D // H)).reshape(B * G, D)
    wt = w.permute(0, 1, 3, 2).reshape(B, H * G, Lp).to(x.dtype)
    full = torch.bmm(wt, x.reshape(B, Lp, D))                                # (B, H*G, H*hd)
    blk = full.view(B, H, G, H, D // H).diagonal(dim1=1, dim2=3)             # (B, G, hd, H)
    return blk.permute(0, 1, 3, 2).reshape(B * G, D)


def _global_rows(gidx, B: int, Lp: int):
    rows = (torch.arange(B, device=gidx.device)[:, None] * Lp + gidx.clamp(min=0).long()).reshape(-1)
    return rows, (gidx >= 0).reshape(-1)


def _attention_torch(q, k, v, qg, h, wkg, bkg, wvg, bvg, flags, gidx, B: int, Lp: int, H: int, half_w: int,
                     drop=None):
    """fp32 recompute of the whole attention block (same contract as the HIP kernels); drop =
    (p, seed) applies attention-probability dropout with the kernels' mask."""
    o = _local_torch(q, k, v, flags, gidx, B, Lp, H, half_w, drop)
    if gidx.shape[1] > 0:
        z = _global_keep(gidx, B, Lp, H, *drop) if drop is not None and drop[0] > 0 else None
        og = _global_torch(qg, h, wkg, bkg, wvg, bvg, flags, B, Lp, H, z)
        rows, keep = _global_rows(gidx, B, Lp)
        # overwrite the valid global rows (TF:621-629) without boolean-mask indexing (a host
        # sync): padded slots point at row 0 of their sequence and add exactly zero
        kf = keep[:, None].to(o.dtype)
        o = o.index_add(0, rows, (og - o[rows]) * kf)
    return o


def _put_global_rows(out, og, rows, keep, B: int, G: int):
    """out[rows[s]] = og[s] for the valid global slots s (TF:621-629), no boolean indexing (a host
    sync): an empty slot rewrites its sequence's first slot row with that slot's own value, so
    repeated rows always receive identical values."""
    r = rows.view(B, G)
    k = keep.view(B, G)
    r0 = r[:, :1].expand(B, G)
    src0 = torch.where(k[:, :1, None], og.view(B, G, -1)[:, :1], out[r[:, 0]].to(og.dtype)[:, None])
    src = torch.where(k[..., None], og.view(B, G, -1), src0.expand(B, G, og.shape[1]))
    out.index_copy_(0, torch.where(k, r, r0).reshape(-1), src.reshape(B * G, -1).to(out.dtype))
    return out


class _Attention(torch.autograd.Function):
    """Takes the fused (B*Lp, 3D) q|k|v projection and returns its gradient as one tensor (no
    per-slice zero-fill + accumulate in autograd). attn_p > 0: attention-probability dropout
    (TF:585-586 local rows on the band kernels, TF:1036-1037 global rows on the fold kernels)
    with the counter-hash mask of `seed`, regenerated in the backward."""

    @staticmethod
    def forward(ctx, qkv, qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, half_w, fold, grows=None,
                attn_p: float = 0.0, seed: int = 0, wkg_master=None, wvg_master=None, wqg16=None, wqgT16=None,
                bqg=None, wqg_master=None, q_scale: float = 1.0, mb=None):
        # mb: a _GradMailbox shared with the q|k|v projection of h (h's gradient from here goes there)
        ctx.mb = mb
        # wkg / wvg: the global key / value weights in the compute dtype; with the masters given
        # (packed copies, not tracked) their gradients go to the fp32 masters directly.
        # wqg16 given (GLOBAL_QG_INSIDE): qg = (h[global rows] Wqg^T + bqg) * q_scale is computed here
        # and its backward runs here too (gradients to bqg and the fp32 master wqg_master)
        ctx.masters = wkg_master is not None
        ctx.qin = wqg16 is not None
        ctx.q_scale = q_scale

        def query_global():
            # the global rows of h (rf_gather_global_rows; an empty slot gathers a zero row, whose
            # qg no output reads)
            hg = ops.gather_global_rows(h, gidx, B, Lp)
            return ops.gemm(hg, wqg16, bqg, ops.RF_EPI_BIAS, scale_cols=qkv.shape[1] // 3, col_scale=q_scale)
        if ctx.qin:
            ctx.qw = (wqg16, wqgT16)
        ctx.fold_ws = None  # the forward fold's workspace when the HIP global backward can use it
        D = qkv.shape[1] // 3
        q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        G = gidx.shape[1]
        ctx.drop = (attn_p, seed) if attn_p > 0 else None
        # the global rows' dropout scale (B, H, G, Lp) fp32 is regenerated in the backward from the
        # seed (ctx.gz_kind), not kept alive on ctx between forward and backward
        ctx.gz_kind = None
        ws = (_fold_ws(h, B, Lp, H, G) if FOLD_SIDE_TRAIN and fold and G > 0 and q.dtype != torch.float32
              and not (ctx.drop is not None and G > 32) else None)
        if ws is not None:
            # the fold's query projection, u and pass over h (stage 1: nothing the local attention reads or
            # writes) on the side stream beside the band kernel; its merge and Wvg (stage 2) after it, into
            # the global rows the band kernel wrote
            def fold_stage1():
                qg1 = query_global() if ctx.qin else qg
                ops.global_attention_fold(qg1.contiguous(), h.contiguous(), wkg.contiguous(), bkg, wvg.contiguous(),
                                          bvg, flags, gidx, B, Lp, H, None, p_drop=attn_p, seed=seed, ws=ws,
                                          stage=1)
                return qg1
            join = _dw_async(fold_stage1, h)
            out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, half_w, p_drop=attn_p, seed=seed)
            qg = join()
            ops.global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, out, p_drop=attn_p, seed=seed,
                                      ws=ws, stage=2)
            ctx.fold_ws = ws
            ctx.gz_kind = "hip" if ctx.drop is not None else None
            ctx.save_for_backward(qkv, qg, h, wkg, bkg, wvg, bvg, flags, gidx, out)
            ctx.dims = (B, Lp, H, half_w)
            ctx.grows = grows
            return out
        if ctx.qin:
            qg = query_global()
        if ctx.drop is not None and q.dtype != torch.float32 and G > 32:
            # the band kernel's dropout form takes <= 32 global keys: recompute in fp32 (the
            # backward of this case is the fp32 recompute as well)
            out = _attention_torch(q, k, v, qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, half_w,
                                   ctx.drop).to(q.dtype)
        elif ctx.drop is not None:
            # global rows under attention dropout (the hash mask) as torch ops; closed-form backward
            out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, half_w, p_drop=attn_p, seed=seed)
            if G > 0 and fold and q.dtype != torch.float32:
                # the fold kernels with the same mask (rf_global_attn_fold_fwd_drop); the mask
                # itself for the closed-form backward from one kernel (rf_attn_global_keep)
                ws = _fold_ws(h, B, Lp, H, G)
                ops.global_attention_fold(qg.contiguous(), h.contiguous(), wkg.contiguous(), bkg,
                                          wvg.contiguous(), bvg, flags, gidx, B, Lp, H, out, p_drop=attn_p, seed=seed,
                                          ws=ws)
                ctx.fold_ws = ws
                ctx.gz_kind = "hip"
            elif G > 0:
                ctx.gz_kind = "torch"
                og = _global_torch(qg, h, wkg, bkg, wvg, bvg, flags, B, Lp, H, _global_keep(gidx, B, Lp, H, attn_p, seed))
                rows, keep = grows[:2] if grows is not None else _global_rows(gidx, B, Lp)
                _put_global_rows(out, og, rows, keep, B, G)
        else:
            out = ops.band_attention(q, k, v, flags, gidx, B, Lp, H, half_w)
        if ctx.drop is None and G > 0:
            if fold:
                ws = _fold_ws(h, B, Lp, H, G) if q.dtype != torch.float32 else None
                ops.global_attention_fold(qg.contiguous(), h.contiguous(), wkg.contiguous(), bkg,
                                          wvg.contiguous(), bvg, flags, gidx, B, Lp, H, out, ws=ws)
                ctx.fold_ws = ws
            else:
                kg = ops.gemm(h.contiguous(), wkg.contiguous(), bkg, ops.RF_EPI_BIAS)
                vg = ops.gemm(h.contiguous(), wvg.contiguous(), bvg, ops.RF_EPI_BIAS)
                ops.global_attention(qg.contiguous(), kg, vg, flags, gidx, B, Lp, H, out)
        ctx.save_for_backward(qkv, qg, h, wkg, bkg, wvg, bvg, flags, gidx, out)
        ctx.dims = (B, Lp, H, half_w)
        ctx.grows = grows  # (rows, keep, rows as int32 with -1 for empty slots) of the pass
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, qg, h, wkg, bkg, wvg, bvg, flags, gidx, out = ctx.saved_tensors
        B, Lp, H, half_w = ctx.dims
        D = qkv.shape[1] // 3
        q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        gmax = gidx.shape[1]
        hip_local = q.dtype in (torch.bfloat16, torch.float16) and half_w == 32 and D == 64 * H and gmax <= 32
        if not hip_local:
            return _Attention._backward_torch(ctx, dout)
        p_drop, seed = ctx.drop if ctx.drop is not None else (0.0, 0)
        # local branch on the HIP backward kernels (rf_attn_bwd.hip); global rows of dout belong
        # to the global branch only (their local output was overwritten)
        d16 = dout.to(q.dtype).contiguous()
        res = [None] * 7
        extra = qtail = None
        need_global = gmax > 0 and (any(ctx.needs_input_grad[1:7]) or any(ctx.needs_input_grad[17:19]) or ctx.qin)
        hip_bwd = GLOBAL_BWD_HIP and ctx.fold_ws is not None
        join_global = None
        if need_global and hip_bwd and GLOBAL_BWD_SIDE:
            # the global rows' backward reads dout, h and the forward's fold workspace only, not the local
            # branch's gradients: its few-block launches run on the side stream beside the local branch's
            # whole-chip kernels (joined before h's gradient is handed on)
            join_global = _dw_async(lambda: _Attention._global_branch(ctx, d16, h, qg, wkg, bkg, wvg, bvg, flags,
                                                                      gidx, B, Lp, H, p_drop, seed, dout, True),
                                    d16)
        # gradients written in the projection's dtype (bf16): no fp32 copy and cast per layer
        dqkv = torch.empty(B * Lp, 3 * D, dtype=qkv.dtype, device=q.device)
        dq, dk, dv, gds, gpr = ops.band_attention_bwd(q, k, v, out, d16, flags, gidx, B, Lp, H, dqkv=dqkv,
                                                      p_drop=p_drop, seed=seed)
        if gmax > 0:
            # gradients of the global-key columns, reduced over every query of the sequence and added
            # into dk / dv at the global positions (bf16, as dqkv)
            if GLOBAL_KV_HIP and gds.shape[-1] == gmax:
                ops.global_kv_grad(gds, gpr, q, d16, gidx, B, Lp, H, dk, dv)
            else:
                rows32 = ctx.grows[2] if ctx.grows is not None else None
                if rows32 is None:
                    rows, keep = _global_rows(gidx, B, Lp)
                    rows32 = torch.where(keep, rows, -1).to(torch.int32)  # -1: empty slot, skipped
                # bf16 operands, fp32 accumulation (no fp32 copies of the (B*Lp, D) q and dout)
                dkg = _global_kv_grad(gds[..., :gmax], q, B, Lp, H)
                dvg = _global_kv_grad(gpr[..., :gmax], d16, B, Lp, H)
                # no boolean-mask indexing (it syncs the host): invalid slots add zeros at row 0
                ops.scatter_add_rows(rows32, dkg.to(dk.dtype).contiguous(), dk, dvg.to(dv.dtype).contiguous(), dv)
            # global branch: closed-form gradient of the fold algebra
            if need_global:
                upd, extra, qtail = (join_global() if join_global is not None else
                                     _Attention._global_branch(ctx, d16, h, qg, wkg, bkg, wvg, bvg, flags, gidx, B,
                                                               Lp, H, p_drop, seed, dout, hip_bwd))
                for n, g in upd.items():
                    res[n] = g
        if ctx.needs_input_grad[0]:
            res[0] = dqkv.to(qkv.dtype)
        tail = [None] * 18  # the forward's non-tensor inputs, the two masters, the query weights, mb
        if extra is not None:
            tail[10:12] = extra
        if qtail is not None:
            tail[12:17] = qtail
        return (*_Attention._post_h(ctx, res, h), *tail)

    @staticmethod
    def _global_branch(ctx, d16, h, qg, wkg, bkg, wvg, bvg, flags, gidx, B: int, Lp: int, H: int, p_drop: float,
                       seed: int, dout, hip_bwd: bool):
        """The global rows' backward (closed form of the fold algebra, or autograd through the torch
        restatement): returns ({input index: gradient} for qg, h, wkg, bkg, wvg, bvg, the fp32 gradients for
        the two key/value masters (or None), the query projection's tail (or None))."""
        gout = gz = None
        if not hip_bwd:
            rows, keep = ctx.grows[:2] if ctx.grows is not None else _global_rows(gidx, B, Lp)
            gout = dout[rows].float() * keep[:, None].to(torch.float32)
        if ctx.gz_kind == "hip" and not hip_bwd:  # the forward's mask, from the same kernel
            gz = ops.attn_global_keep(gidx, B, Lp, H, p_drop, seed)
        elif ctx.gz_kind == "torch":
            gz = _global_keep(gidx, B, Lp, H, p_drop, seed)
        if hip_bwd:
            with torch.autocast("cuda", enabled=False):
                grads = _global_bwd_hip(qg, h, wkg, wvg, bvg, flags, gidx, B, Lp, H, d16, ctx.fold_ws, p_drop, seed)
        elif GLOBAL_BWD_CLOSED_FORM:
            with torch.autocast("cuda", enabled=False):
                grads = _global_bwd(qg, h, wkg, wvg, flags, B, Lp, H, gout, gz, bvg,
                                    dh_dtype=h.dtype if GLOBAL_BWD_DH16 else None)
        else:
            gin = [t.detach().requires_grad_(True) for t in (qg, h, wkg, bkg, wvg, bvg)]
            with torch.enable_grad(), torch.autocast("cuda", enabled=False):
                og = _global_torch(*gin, flags, B, Lp, H, gz)
                grads = torch.autograd.grad(og, gin, gout, allow_unused=True)
        upd = {}
        for n, t in enumerate((qg, h, wkg, bkg, wvg, bvg)):
            if ctx.needs_input_grad[1 + n] or (n == 1 and ctx.qin):
                g = grads[n]
                upd[1 + n] = None if g is None else g.to(t.dtype)
        extra = qtail = None
        if ctx.masters:  # fp32 gradients straight to the masters (no bf16 round trip)
            extra = [grads[2].float() if ctx.needs_input_grad[17] and grads[2] is not None else None,
                     grads[4].float() if ctx.needs_input_grad[18] and grads[4] is not None else None]
        if ctx.qin:
            upd[2], qtail = _Attention._qg_backward(ctx, grads[0], upd.get(2), h, gidx, B, Lp, hip_bwd)
        return upd, extra, qtail

    @staticmethod
    def _post_h(ctx, res, h):
        """h's gradient into the mailbox (the q|k|v projection's dA adds it) instead of to autograd."""
        dh = res[2]
        if (ctx.mb is not None and dh is not None and dh.dtype == h.dtype and dh.shape == h.shape
                and dh.is_contiguous()):
            ctx.mb.g = dh
            res = list(res)
            res[2] = None
        return res

    @staticmethod
    def _qg_backward(ctx, dqg, dh, h, gidx, B: int, Lp: int, hip: bool):
        """Backward of the query_global projection computed in the forward (GLOBAL_QG_INSIDE): returns
        (h's gradient with the global rows' part added, the tail for (wqg16, wqgT16, bqg, wqg_master,
        q_scale)). HIP: rf_global_query_bwd in place into dh; else torch."""
        wqg16, wqgT16 = ctx.qw
        s = ctx.q_scale
        if dh is None:
            dh = torch.zeros_like(h)
        if hip and dh.dtype == h.dtype and dh.is_contiguous() and wqgT16.is_contiguous():
            dwqg, dbqg = ops.global_query_bwd(gidx, dqg.float().contiguous(), s, h, wqgT16, dh, B, Lp)
        else:
            rows, keep = _global_rows(gidx, B, Lp)
            dqs = dqg.float() * s * keep[:, None].to(torch.float32)
            hg = h.index_select(0, rows).float()
            dwqg = dqs.t() @ hg
            dbqg = dqs.sum(0)
            dh = dh.index_add(0, rows, (dqs @ wqg16.float()).to(dh.dtype))
        return dh, [None, None, dbqg if ctx.needs_input_grad[21] else None,
                    dwqg if ctx.needs_input_grad[22] else None, None]

    @staticmethod
    def _backward_torch(ctx, dout):
        qkv, qg, h, wkg, bkg, wvg, bvg, flags, gidx, _ = ctx.saved_tensors
        B, Lp, H, half_w = ctx.dims
        D = qkv.shape[1] // 3
        need = list(ctx.needs_input_grad)
        if ctx.masters:  # gradients of the packed copies go to the masters
            need[3] = need[3] or need[17]
            need[5] = need[5] or need[18]
        if ctx.qin:  # qg was computed in the forward: its gradient feeds the projection's backward
            need[1] = need[2] = True
        inputs = [t.detach().requires_grad_(nd) for t, nd in
                  zip((qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], qg, h, wkg, bkg, wvg, bvg),
                      (need[0],) * 3 + tuple(need[1:7]))]
        with torch.enable_grad(), torch.autocast("cuda", enabled=False):
            o = _attention_torch(*inputs, flags, gidx, B, Lp, H, half_w, ctx.drop)
            want = [t for t in inputs if t.requires_grad]
            grads = torch.autograd.grad(o, want, dout.float(), allow_unused=True) if want else []
        it = iter(grads)
        res = []
        for t in inputs:
            if t.requires_grad:
                g = next(it)
                res.append(None if g is None else g.to(t.dtype))
            else:
                res.append(None)
        if need[0]:
            z = [g if g is not None else torch.zeros_like(qkv[:, :D]) for g in res[:3]]
            res = [torch.cat(z, 1)] + res[3:]
        else:
            res = [None] + res[3:]
        tail = [None] * 18  # the forward's non-tensor inputs, the two masters, the query weights, mb
        if ctx.masters:
            g_k, g_v = res[3], res[5]
            res[3] = res[5] = None
            tail[10:12] = [None if g_k is None else g_k.float(), None if g_v is None else g_v.float()]
        if ctx.qin and gidx.shape[1] > 0:
            dqg = res[1] if res[1] is not None else torch.zeros_like(qg, dtype=torch.float32)
            res[1] = None
            B, Lp = ctx.dims[0], ctx.dims[1]
            res[2], tail[12:17] = _Attention._qg_backward(ctx, dqg, res[2], h, gidx, B, Lp, False)
        return (*_Attention._post_h(ctx, res, h), *tail)


# ------------------------------------------------------------------------------------------
# Global-slot count of a captured training step (set by recformer_amd.graphs while capturing and
# replaying): encode_train then takes it instead of reading max(#global tokens) back from the device.
_STATIC_GMAX: Optional[int] = None


# ------------------------------------------------------------------------------------------
# Per-forward cache of the autograd-tracked weight casts (bf16 copies, the fused q|k|v weight):
# RecformerForPretraining runs four encoder passes over the same parameters, and one cast node
# per parameter shared by all four (gradients accumulate through it) replaces four.
_CASTS: Optional[dict] = None


class shared_casts:
    """Context manager: within it, encode_train reuses each weight cast it has made."""

    def __enter__(self):
        global _CASTS
        self._outer = _CASTS
        if _CASTS is None:
            _CASTS = {}
        return self

    def __exit__(self, *exc):
        global _CASTS
        _CASTS = self._outer
        return False


def _cast(key, make):
    if _CASTS is None:
        return make()
    t = _CASTS.get(key)
    if t is None:
        t = _CASTS[key] = make()
    return t


def _layer_weights(li: int, lyr, dt: torch.dtype) -> dict:
    """The layer's weights as the forward consumes them (cached under shared_casts): each GEMM
    weight as (master, untracked compute-dtype copy) for _Gemm; the global key/value weights as
    tracked casts (the attention backward returns their gradients in the compute dtype)."""
    def make():
        sa, ao, fo = lyr.attention.self, lyr.attention.output, lyr.output

        def pair(w):
            return w, w.detach().to(dt)
        return {
            "w_qkv": pair(torch.cat([sa.query.weight, sa.key.weight, sa.value.weight], 0)),
            "b_qkv": torch.cat([sa.query.bias, sa.key.bias, sa.value.bias], 0).float(),
            "w_qg": pair(sa.query_global.weight), "b_qg": sa.query_global.bias.float(),
            "w_kg": sa.key_global.weight.to(dt), "b_kg": sa.key_global.bias.float(),
            "w_vg": sa.value_global.weight.to(dt), "b_vg": sa.value_global.bias.float(),
            "w_o": pair(ao.dense.weight), "b_o": ao.dense.bias.float(),
            "w_1": pair(lyr.intermediate.dense.weight), "b_1": lyr.intermediate.dense.bias.float(),
            "w_2": pair(fo.dense.weight), "b_2": fo.dense.bias.float(),
        }
    return _cast((id(lyr), li, dt), make)


# One rf_pack_weights launch per forward writes every encoder GEMM weight's compute-dtype copy and
# its transposed copy (ops.WeightPack, persistent buffers per model and dtype) — instead of a cast,
# a q|k|v concatenation and, in the backward, a transpose (+ scaled clone) per weight per step.
PACK_WEIGHTS = True
_PACKS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _pack_sources(model):
    out = []
    for lyr in model.encoder.layer:
        sa = lyr.attention.self
        out += [sa.query.weight, sa.key.weight, sa.value.weight, sa.query_global.weight,
                lyr.attention.output.dense.weight, lyr.intermediate.dense.weight, lyr.output.dense.weight,
                sa.key_global.weight, sa.value_global.weight]
    return out


def _encoder_pack(model, dt: torch.dtype, scale: float):
    """(pack, per-layer buffers) for the model's current weights, (re)built when they moved."""
    srcs = _pack_sources(model)
    per = _PACKS.setdefault(model, {})
    ent = per.get(dt)
    if ent is not None and ent[2] == scale and ent[0].ptrs == tuple(w.data_ptr() for w in srcs):
        return ent
    layers, specs = [], []
    for li, lyr in enumerate(model.encoder.layer):
        q, k, v, qg, o, f1, f2, kg, vg = (w.detach() for w in srcs[9 * li:9 * li + 9])
        D, Fd = q.shape[1], f1.shape[0]

        def e(*shape):
            return torch.empty(*shape, dtype=dt, device=q.device)
        bufs = {"qkv": (e(3 * D, D), e(D, 3 * D)), "qg": (e(D, D), e(D, D)), "o": (e(D, D), e(D, D)),
                "f1": (e(Fd, D), e(D, Fd)), "f2": (e(D, Fd), e(Fd, D)), "kg": e(D, D), "vg": e(D, D)}
        qb, qt = bufs["qkv"]
        specs += [dict(src=q, dst=(qb, 0), dstT=(qt, 0), scale_n=D, t_scale=scale),
                  dict(src=k, dst=(qb, D), dstT=(qt, D)), dict(src=v, dst=(qb, 2 * D), dstT=(qt, 2 * D)),
                  dict(src=qg, dst=(bufs["qg"][0], 0), dstT=(bufs["qg"][1], 0), scale_n=D, t_scale=scale),
                  dict(src=o, dst=(bufs["o"][0], 0), dstT=(bufs["o"][1], 0)),
                  dict(src=f1, dst=(bufs["f1"][0], 0), dstT=(bufs["f1"][1], 0)),
                  dict(src=f2, dst=(bufs["f2"][0], 0), dstT=(bufs["f2"][1], 0)),
                  dict(src=kg, dst=(bufs["kg"], 0)), dict(src=vg, dst=(bufs["vg"], 0))]
        layers.append(bufs)
    ent = (ops.WeightPack(specs, dt), layers, scale)
    per[dt] = ent
    return ent


def _packed_layer_weights(model, dt: torch.dtype, scale: float):
    """Per-layer weights for the packed path, the pack refreshed once per forward (once per step
    under shared_casts, the four pretraining passes)."""
    def make():
        pack, layers, _ = _encoder_pack(model, dt, scale)
        pack.refresh()
        out = []
        for lyr, bufs in zip(model.encoder.layer, layers):
            sa, ao, fo = lyr.attention.self, lyr.attention.output, lyr.output
            out.append({
                "packed": True,
                "w_qkv": ((sa.query.weight, sa.key.weight, sa.value.weight),) + bufs["qkv"],
                "b_qkv": torch.cat([sa.query.bias, sa.key.bias, sa.value.bias], 0).float(),
                "w_qg": ((sa.query_global.weight,),) + bufs["qg"], "b_qg": sa.query_global.bias.float(),
                "w_kg": bufs["kg"], "b_kg": sa.key_global.bias.float(), "wkg_master": sa.key_global.weight,
                "w_vg": bufs["vg"], "b_vg": sa.value_global.bias.float(), "wvg_master": sa.value_global.weight,
                "w_o": ((ao.dense.weight,),) + bufs["o"], "b_o": ao.dense.bias.float(),
                "w_1": ((lyr.intermediate.dense.weight,),) + bufs["f1"], "b_1": lyr.intermediate.dense.bias.float(),
                "w_2": ((fo.dense.weight,),) + bufs["f2"], "b_2": fo.dense.bias.float(),
            })
        return out
    return _cast(("pack", id(model), dt, scale), make)


def _lin(a, lw, wkey: str, bkey: str, scale_cols: int, col_scale: float, mb=None):
    """One of the layer's Linears: _GemmP over the packed weights (mb: a _GradMailbox through which
    another consumer of `a` hands over its gradient), or _Gemm (master, w16)."""
    if lw.get("packed"):
        masters, w16, w16t = lw[wkey]
        return _GemmP.apply(a, lw[bkey], w16, w16t, scale_cols, col_scale, mb, *masters)
    return _Gemm.apply(a, *lw[wkey], lw[bkey], scale_cols, col_scale)


class _GlobalCLS(torch.autograd.Function):
    """The last layer's attention output at the B CLS rows only (encode_train with pooled_only; the
    training form of models._cls_last_layer): the global rows through the fold kernels (with the
    attention-dropout mask of `seed`), the CLS rows returned; backward = rf_global_fold_bwd_full with
    the CLS rows' gradient (nothing reads the other rows, so their gradient is zero) — no qkv GEMM and
    no band attention either way. Inputs (qg, h, wkg, bkg, wvg, bvg) as _Attention's global part; with
    the fp32 masters given, the key / value weight gradients go to them."""

    @staticmethod
    def forward(ctx, qg, h, wkg, bkg, wvg, bvg, flags, gidx, B, Lp, H, attn_p, seed, ws, wkg_master=None,
                wvg_master=None):
        D = h.shape[1]
        out = torch.empty(B * Lp, D, dtype=h.dtype, device=h.device)
        ops.global_attention_fold(qg.contiguous(), h.contiguous(), wkg.contiguous(), bkg, wvg.contiguous(), bvg,
                                  flags, gidx, B, Lp, H, out, p_drop=attn_p, seed=seed, ws=ws)
        rows = torch.arange(B, device=h.device) * Lp
        ctx.save_for_backward(qg, h, wkg, wvg, bvg, flags, gidx, rows)
        ctx.meta = (B, Lp, H, attn_p, seed, ws, wkg_master is not None)
        return out.index_select(0, rows)

    @staticmethod
    def backward(ctx, dcls):
        qg, h, wkg, wvg, bvg, flags, gidx, rows = ctx.saved_tensors
        B, Lp, H, p, seed, ws, masters = ctx.meta
        d16 = torch.zeros(B * Lp, h.shape[1], dtype=h.dtype, device=h.device)
        d16.index_copy_(0, rows, dcls.to(h.dtype))
        with torch.autocast("cuda", enabled=False):
            dqg, dh, dwkg, dbkg, dwvg, dbvg = _global_bwd_hip(qg, h, wkg, wvg, bvg, flags, gidx, B, Lp, H, d16,
                                                              ws, p, seed)
        need = ctx.needs_input_grad
        res = [dqg.to(qg.dtype) if need[0] else None, dh.to(h.dtype) if need[1] else None,
               None if masters or not need[2] else dwkg.to(wkg.dtype), dbkg if need[3] else None,
               None if masters or not need[4] else dwvg.to(wvg.dtype), dbvg if need[5] else None]
        tail = [None] * 10  # flags, gidx, B, Lp, H, attn_p, seed, ws, then the two masters
        if masters:
            tail[8] = dwkg.float() if need[14] else None
            tail[9] = dwvg.float() if need[15] else None
        return (*res, *tail)


class _ZeroGrads(torch.autograd.Function):
    """Identity on x whose backward also gives the listed parameters an all-zero gradient: the last
    layer's local query / key / value projections do not reach the CLS rows (their gradient in the full
    layer is exactly zero), and the optimizer must see a zero gradient — not None — to apply weight
    decay to them as it does after the full layer's backward."""

    @staticmethod
    def forward(ctx, x, *params):
        ctx.shapes = [(p.shape, p.dtype, p.device) for p in params]
        return x.view_as(x)

    @staticmethod
    def backward(ctx, dx):
        return (dx, *[torch.zeros(s, dtype=d, device=dv) for s, d, dv in ctx.shapes])


# the CLS-global flag of a captured step's example batch (recformer_amd.graphs), as _STATIC_GMAX
_STATIC_CLS: Optional[bool] = None


def encode_train(model, input_ids, attention_mask, global_attention_mask, token_type_ids,
                 position_ids, item_position_ids, output_hidden_states: bool, word=None, head_cols=None,
                 attn_probe=None, pooled_only: bool = False) -> Tuple[torch.Tensor, Optional[tuple]]:
    """Autograd forward of RecformerModel (same outputs as RecformerModel._encode). `word` replaces the
    word-embedding table (inputs_embeds, models._embeds_as_table); `head_cols` (layers, hidden) scales
    each layer's attention context (head_mask, models._head_mask_columns); `attn_probe`, a list, receives
    each layer's (attentions, global_attentions) (output_attentions, recformer_amd/probs.py). With
    `pooled_only` (RecformerForSeqRec: the loss reads the CLS rows only) and every CLS a global token,
    the last layer runs on the CLS rows (_GlobalCLS) and (pooled (B, d) fp32, None) is returned, with
    model._last_pruned set."""
    model._last_pruned = False
    from .models import _compute_dtype
    cfg = model.config
    B, L = input_ids.shape
    Wn = model._window()
    Lp = L + (Wn - L % Wn) % Wn
    D, H = cfg.hidden_size, cfg.num_attention_heads
    hd = D // H
    dt = _compute_dtype(model.dtype)
    eps = cfg.layer_norm_eps
    p_hid = cfg.hidden_dropout_prob if model.training else 0.0
    p_att = cfg.attention_probs_dropout_prob if model.training else 0.0
    if global_attention_mask is not None:
        gm = global_attention_mask != 0
        if attention_mask is not None:
            gm = gm & (attention_mask > 0)
        # a captured step (recformer_amd.graphs) fixes the global-slot count: no host sync, empty slots
        # (gidx < 0) are inert
        gmax = _STATIC_GMAX if _STATIC_GMAX is not None else (int(gm.sum(1).max().item()) if B > 0 else 0)
        from . import models as _models
        want = pooled_only and _models.PRUNE_LAST_LAYER and cfg.pooler_type == "cls" and not output_hidden_states \
            and attn_probe is None and B > 0
        if not want:
            cls_global = False
        elif _STATIC_GMAX is not None:
            cls_global = bool(_STATIC_CLS)
        else:
            cls_global = bool(gm[:, 0].all())
    else:
        gmax = 0
        cls_global = False
    ids, pos, tt, ip, flags, gidx = ops.prepare_inputs(
        input_ids, attention_mask, global_attention_mask, token_type_ids, item_position_ids,
        position_ids, Lp, cfg.pad_token_id, gmax)
    emb = model.embeddings
    h32 = _EmbedLN.apply(ids, pos, tt, ip, emb.word_embeddings.weight.float() if word is None else word,
                         emb.position_embeddings.weight.float(), emb.token_type_embeddings.weight.float(),
                         emb.item_position_embeddings.weight.float(), emb.LayerNorm.weight.float(),
                         emb.LayerNorm.bias.float(), eps, cfg.pad_token_id)
    h32 = F.dropout(h32, p_hid, model.training)
    hidden_all = [h32] if output_hidden_states else None
    scale = 1.0 / math.sqrt(hd)
    windows = cfg.window_per_layer()
    fold = getattr(cfg, "global_attention_fold", True)
    rows = grows = None
    if gmax > 0:
        rows = (torch.arange(B, device=input_ids.device)[:, None] * Lp + gidx.clamp(min=0).long()).reshape(-1)
        gvalid = (gidx >= 0).reshape(-1, 1)
        grows = (rows, gvalid.view(-1), torch.where(gvalid.view(-1), rows, -1).to(torch.int32))
    # bf16 path: dropout + residual + LayerNorm as one HIP pass each way (_DropAddLN)
    fused = dt in (torch.bfloat16, torch.float16) and D in (64, 128, 256, 384, 512, 768, 1024)
    h16 = None  # bf16 copy of h32 written by the previous layer's LayerNorm (fused path)
    nl = len(model.encoder.layer)
    # the pass's dropout seeds (two LayerNorms per layer) in one draw from torch's CPU generator
    seeds = torch.randint(0, 2 ** 62, (2 * nl,)).tolist() if p_hid > 0 else [0] * (2 * nl)
    att_seeds = torch.randint(0, 2 ** 62, (nl,)).tolist() if p_att > 0 else [0] * nl
    packed = None
    if PACK_WEIGHTS and fused and FFN_FUSED and D % 64 == 0 and cfg.intermediate_size % 64 == 0 and input_ids.is_cuda:
        packed = _packed_layer_weights(model, dt, scale)
    # query_global projection inside _Attention when its backward takes the HIP global path (the fold
    # workspace's limits, the HIP local backward's window)
    qg_inside = (GLOBAL_QG_INSIDE and GLOBAL_BWD_HIP and packed is not None and gmax <= 4 and fold and
                 D % 128 == 0 and D <= 768 and D == 64 * H and B * gmax <= 1024 and
                 all(w == 64 for w in windows))
    for li, lyr in enumerate(model.encoder.layer):
        lw = packed[li] if packed is not None else _layer_weights(li, lyr, dt)
        h = h16 if h16 is not None else h32.to(dt)
        if li == nl - 1 and cls_global and fold and fused and gmax > 0 and h.is_cuda:
            ws = _fold_ws(h, B, Lp, H, gmax)
            if ws is not None:
                model._last_pruned = True
                return _cls_last_layer_train(model, lyr, lw, h, h32, rows, gvalid, flags, gidx, B, Lp, H, D, dt,
                                             scale, eps, p_hid, p_att, seeds[2 * li:2 * li + 2], att_seeds[li], ws,
                                             head_cols, li), None
        if attn_probe is not None:
            from .probs import layer_attention_probs
            attn_probe.append(layer_attention_probs(
                h.detach(), lyr.attention.self, flags, gidx, B, Lp, L, Lp, H, windows[li] // 2, scale,
                None if head_cols is None else head_cols[li, ::hd].detach()))
        # the attention's gradient of h joins the q|k|v projection's dA in its epilogue (packed weights,
        # 16-bit h: the residual form of the GEMM)
        mb = _GradMailbox() if (lw.get("packed") and GRAD_MAILBOX and h.dtype != torch.float32) else None
        qkv = _lin(h, lw, "w_qkv", "b_qkv", D, scale, mb)
        qg = None
        qin = ()
        if gmax > 0 and qg_inside:
            (wqg_m,), wqg16, wqgT16 = lw["w_qg"]
            qin = (wqg16, wqgT16, lw["b_qg"], wqg_m, scale)
        elif gmax > 0:
            hg = h[rows] * gvalid.to(h.dtype)
            qg = _lin(hg, lw, "w_qg", "b_qg", D, scale)
        ctx = _Attention.apply(qkv, qg, h, lw["w_kg"], lw["b_kg"], lw["w_vg"], lw["b_vg"],
                               flags, gidx, B, Lp, H, windows[li] // 2, fold, grows, p_att, att_seeds[li],
                               lw.get("wkg_master"), lw.get("wvg_master"), *(qin or (None, None, None, None, 1.0)), mb)
        if head_cols is not None:
            ctx = ctx * head_cols[li].to(ctx.dtype)
        ao = lyr.attention.output
        t = _lin(ctx, lw, "w_o", "b_o", 0, 1.0)
        if fused:
            a32, a16 = _DropAddLN.apply(t, h32, ao.LayerNorm.weight, ao.LayerNorm.bias, eps, p_hid, True,
                                        seeds[2 * li])
        else:
            x1 = F.dropout(t.float(), p_hid, model.training) + h32
            a32 = _LayerNorm.apply(x1, ao.LayerNorm.weight.float(), ao.LayerNorm.bias.float(), eps, torch.float32)
            a16 = a32.to(dt)
        fo = lyr.output
        if lw.get("packed"):
            (w1,), w1_16, w1t = lw["w_1"]
            (w2,), w2_16, w2t = lw["w_2"]
            t2 = _FFN.apply(a16, w1, w1_16, lw["b_1"], w2, w2_16, lw["b_2"], w1t, w2t)
        elif fused and FFN_FUSED and D % 64 == 0 and lw["w_1"][1].shape[0] % 64 == 0:
            t2 = _FFN.apply(a16, *lw["w_1"], lw["b_1"], *lw["w_2"], lw["b_2"])
        else:
            if dt == torch.bfloat16 and FUSED_GELU:
                u = _GemmGelu.apply(a16, *lw["w_1"], lw["b_1"])
            else:
                u = F.gelu(_Gemm.apply(a16, *lw["w_1"], lw["b_1"], 0, 1.0))
            t2 = _Gemm.apply(u, *lw["w_2"], lw["b_2"], 0, 1.0)
        if fused and li + 1 < nl:
            h32, h16 = _DropAddLN.apply(t2, a32, fo.LayerNorm.weight, fo.LayerNorm.bias, eps, p_hid, True,
                                        seeds[2 * li + 1])
        elif fused:
            h32 = _DropAddLN.apply(t2, a32, fo.LayerNorm.weight, fo.LayerNorm.bias, eps, p_hid, False,
                                   seeds[2 * li + 1])
        else:
            x2 = F.dropout(t2.float(), p_hid, model.training) + a32
            h32 = _LayerNorm.apply(x2, fo.LayerNorm.weight.float(), fo.LayerNorm.bias.float(), eps, torch.float32)
        if output_hidden_states:
            hidden_all.append(h32)
    last = h32.view(B, Lp, D)[:, :L]
    if output_hidden_states:
        hidden_all = tuple(x.view(B, Lp, D)[:, :L] for x in hidden_all)
    return last, hidden_all


def _cls_last_layer_train(model, lyr, lw, h, h32, rows, gvalid, flags, gidx, B: int, Lp: int, H: int, D: int, dt,
                          scale: float, eps: float, p_hid: float, p_att: float, seeds, att_seed: int, ws, head_cols,
                          li: int) -> torch.Tensor:
    """encode_train's last layer on the CLS rows (see _GlobalCLS): query_global on the global rows,
    the fold at the CLS rows, then the output projection, residual LayerNorms and FFN on B rows.
    Returns the pooled vectors (B, d) fp32 (differentiable)."""
    hg = h[rows] * gvalid.to(h.dtype)
    qg = _lin(hg, lw, "w_qg", "b_qg", D, scale)
    c = _GlobalCLS.apply(qg, h, lw["w_kg"], lw["b_kg"], lw["w_vg"], lw["b_vg"], flags, gidx, B, Lp, H, p_att,
                         att_seed, ws, lw.get("wkg_master"), lw.get("wvg_master"))
    if head_cols is not None:
        c = c * head_cols[li].to(c.dtype)
    cls = torch.arange(B, device=h.device) * Lp
    res = h32.index_select(0, cls)
    ao, fo = lyr.attention.output, lyr.output
    t = _lin(c, lw, "w_o", "b_o", 0, 1.0)
    # the compacted CLS rows draw the hidden-dropout masks of their full-layer rows b * Lp
    a32, a16 = _DropAddLN.apply(t, res, ao.LayerNorm.weight, ao.LayerNorm.bias, eps, p_hid, True, seeds[0], Lp)
    if lw.get("packed"):
        (w1,), w1_16, w1t = lw["w_1"]
        (w2,), w2_16, w2t = lw["w_2"]
        t2 = _FFN.apply(a16, w1, w1_16, lw["b_1"], w2, w2_16, lw["b_2"], w1t, w2t)
    elif FFN_FUSED and D % 64 == 0 and lw["w_1"][1].shape[0] % 64 == 0:
        t2 = _FFN.apply(a16, *lw["w_1"], lw["b_1"], *lw["w_2"], lw["b_2"])
    else:
        if dt == torch.bfloat16 and FUSED_GELU:
            u = _GemmGelu.apply(a16, *lw["w_1"], lw["b_1"])
        else:
            u = F.gelu(_Gemm.apply(a16, *lw["w_1"], lw["b_1"], 0, 1.0))
        t2 = _Gemm.apply(u, *lw["w_2"], lw["b_2"], 0, 1.0)
    y = _DropAddLN.apply(t2, a32, fo.LayerNorm.weight, fo.LayerNorm.bias, eps, p_hid, False, seeds[1], Lp)
    sa = lyr.attention.self
    local = [p for m in (sa.query, sa.key, sa.value) for p in (m.weight, m.bias) if p.requires_grad]
    return _ZeroGrads.apply(y, *local) if local else y
