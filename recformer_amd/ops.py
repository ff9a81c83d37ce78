"""Tensor-level wrappers over the C ABI (include/recformer_hip.h).

Each function takes torch tensors that already live on a ROCm device, validates shape /
dtype / contiguity on the host, and launches on torch's current stream. Buffers are
allocated by PyTorch's caching allocator; the library never allocates or syncs.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from ._lib import (RF_BF16, RF_EPI_BIAS, RF_EPI_BIAS_GELU, RF_EPI_BIAS_GELU_AUX, RF_EPI_BIAS_RESID, RF_EPI_COS,
                   RF_EPI_DGELU,
                   RF_EPI_NONE, RF_F32, check)

__all__ = [
    "dtype_code", "prepare_inputs", "embed_ln", "embed_ln_split", "add_layernorm_split", "join_split",
    "gemm", "weight_grad", "WeightPack", "embed_ln_bwd", "embedding_grad", "colsum", "layernorm", "layernorm_bwd", "drop_add_ln_fwd", "drop_add_ln_bwd", "add_layernorm", "band_attention_bwd", "band_attention",
    "global_attention", "gather_global_rows", "row_inv_norm", "cos_scores", "cos_scores_cand",
    "cross_entropy",
    "cos_scores_bwd",
    "RF_EPI_NONE", "RF_EPI_BIAS", "RF_EPI_BIAS_GELU", "RF_EPI_BIAS_GELU_AUX", "RF_EPI_BIAS_RESID", "RF_EPI_COS",
    "RF_EPI_DGELU",
]


# ---- optional per-launch timing (bench.py): HIP events recorded on the launch stream ----
_TIMING: Optional[Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event]]]] = None


def enable_timing(on: bool = True) -> None:
    global _TIMING
    _TIMING = {} if on else None


def timing_results() -> Dict[str, List[float]]:
    """Per-tag launch durations in ms (synchronises)."""
    if not _TIMING:
        return {}
    torch.cuda.synchronize()
    return {k: [s.elapsed_time(e) for s, e in v] for k, v in _TIMING.items()}


@contextlib.contextmanager
def _region(tag: Optional[str]):
    if _TIMING is None or tag is None:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _TIMING.setdefault(tag, []).append((s, e))


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return RF_BF16
    if dt == torch.float32:
        return RF_F32
    if dt == torch.float16:
        return _lib.RF_F16
    raise TypeError(f"recformer_amd: unsupported compute dtype {dt} (bf16, fp16 or fp32)")


def _dev(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.RecformerHipError(
                "recformer_amd kernels need ROCm device tensors (no CPU fallback); got a CPU tensor")


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _rowmajor(t: torch.Tensor, name: str) -> int:
    """Leading dimension of a 2-D row-major view (unit column stride)."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D row-major tensor, got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")
    return t.stride(0)


def prepare_inputs(input_ids, attention_mask, global_attention_mask, token_type_ids,
                   item_position_ids, position_ids, Lp: int, pad_id: int, gmax: int,
                   gstat: Optional[torch.Tensor] = None):
    """A2 prologue (models.py:306-329). Returns int32 ids/pos/tt/ip (B,Lp), uint8 flags,
    int32 gidx (B,gmax). gstat: an int32 (B, 2) tensor to receive each sequence's global-token count
    and whether its position 0 is global (from the same pass)."""
    lib = _lib.load()
    _dev(input_ids)
    B, L = input_ids.shape
    dev = input_ids.device

    def i64(t):
        if t is None:
            return None
        _dev(t)
        if t.shape != (B, L):
            raise ValueError(f"input of shape {tuple(t.shape)} does not match input_ids {(B, L)}")
        return t.to(torch.int64).contiguous()

    ids_in = i64(input_ids)
    am, gm, tt_in, ip_in, pos_in = (i64(attention_mask), i64(global_attention_mask),
                                    i64(token_type_ids), i64(item_position_ids), i64(position_ids))
    if ip_in is None:
        raise ValueError("item_position_ids is required (RecformerEmbeddings, models.py:132)")
    ids = torch.empty(B, Lp, dtype=torch.int32, device=dev)
    pos = torch.empty_like(ids)
    tt = torch.empty_like(ids)
    ip = torch.empty_like(ids)
    flags = torch.empty(B, Lp, dtype=torch.uint8, device=dev)
    gidx = torch.empty(B, max(gmax, 1), dtype=torch.int32, device=dev)
    if gstat is not None and (gstat.dtype != torch.int32 or tuple(gstat.shape) != (B, 2) or not gstat.is_contiguous()):
        raise ValueError("prepare_inputs: gstat must be a contiguous int32 (B, 2) tensor")
    check(lib.rf_prepare_inputs(_p(ids_in), _p(am), _p(gm), _p(tt_in), _p(ip_in), _p(pos_in), B, L,
                                Lp, pad_id, gmax, _p(ids), _p(pos), _p(tt), _p(ip), _p(flags),
                                _p(gidx), _p(gstat), _stream(ids)), "rf_prepare_inputs")
    return ids, pos, tt, ip, flags, gidx[:, :gmax]


def embed_ln(ids, pos, tt, ip, word, posemb, typeemb, iposemb, ln_w, ln_b, eps: float,
             out_dtype: Optional[torch.dtype] = None, want_f32: bool = False):
    """Returns (out in out_dtype, fp32 copy or None)."""
    lib = _lib.load()
    _dev(ids, word)
    M = ids.numel()
    D = word.shape[1]
    for t in (word, posemb, typeemb, iposemb):
        if not t.is_contiguous() or t.dtype != word.dtype or t.shape[1] != D:
            raise ValueError("embedding tables must be contiguous, same dtype and width")
    odt = out_dtype or word.dtype
    out = torch.empty(M, D, dtype=odt, device=word.device)
    out32 = torch.empty(M, D, dtype=torch.float32, device=word.device) if want_f32 else None
    check(lib.rf_embed_ln_fwd(dtype_code(word.dtype), dtype_code(odt), M, D, _p(ids), _p(pos), _p(tt),
                              _p(ip), _p(word), _p(posemb), _p(typeemb), _p(iposemb),
                              _p(ln_w.float().contiguous()), _p(ln_b.float().contiguous()),
                              float(eps), _p(out), _p(out32), _stream(out)), "rf_embed_ln_fwd")
    return out, out32


def embed_ln_split(ids, pos, tt, ip, word, posemb, typeemb, iposemb, ln_w, ln_b, eps: float):
    """The embedding LayerNorm output as the split fp32 stream: (hi bf16, lo int16) planes
    (rf_embed_ln_split_fwd; hi is the first layer's GEMM operand)."""
    lib = _lib.load()
    _dev(ids, word)
    M = ids.numel()
    D = word.shape[1]
    for t in (word, posemb, typeemb, iposemb):
        if not t.is_contiguous() or t.dtype != word.dtype or t.shape[1] != D:
            raise ValueError("embedding tables must be contiguous, same dtype and width")
    hi = torch.empty(M, D, dtype=torch.bfloat16, device=word.device)
    lo = torch.empty(M, D, dtype=torch.int16, device=word.device)
    check(lib.rf_embed_ln_split_fwd(dtype_code(word.dtype), M, D, _p(ids), _p(pos), _p(tt), _p(ip),
                                    _p(word), _p(posemb), _p(typeemb), _p(iposemb),
                                    _p(ln_w.float().contiguous()), _p(ln_b.float().contiguous()),
                                    float(eps), _p(hi), _p(lo), _stream(hi)), "rf_embed_ln_split_fwd")
    return hi, lo


def add_layernorm_split(x: torch.Tensor, res_hi: torch.Tensor, res_lo: torch.Tensor, w: torch.Tensor,
                        b: torch.Tensor, eps: float, planes: bool = True, want_f32: bool = False,
                        tag: Optional[str] = None):
    """y = LN(x + r) on the split fp32 stream (rf_add_layernorm_split_fwd): x the bf16 dense output,
    r = join(res_hi, res_lo). With `planes` the new stream overwrites (res_hi, res_lo) in place;
    `want_f32` also returns an fp32 copy. Returns (hi, lo, y32) (entries None when not written)."""
    lib = _lib.load()
    _dev(x, res_hi, res_lo)
    M, D = x.shape
    if x.dtype != torch.bfloat16:
        raise TypeError("add_layernorm_split: x must be bf16")
    for t, dt in ((res_hi, torch.bfloat16), (res_lo, torch.int16)):
        if t.dtype != dt or not t.is_contiguous() or tuple(t.shape) != (M, D):
            raise ValueError("add_layernorm_split: residual planes must be contiguous (M, D) bf16 / int16")
    if not (planes or want_f32):
        raise ValueError("add_layernorm_split: no output requested")
    y32 = torch.empty(M, D, dtype=torch.float32, device=x.device) if want_f32 else None
    yh, yl = (res_hi, res_lo) if planes else (None, None)
    with _region(tag):
        rc = lib.rf_add_layernorm_split_fwd(M, D, _p(x), _rowmajor(x, "x"), _p(res_hi), _p(res_lo),
                                            _p(w), _p(b), float(eps), _p(yh), _p(yl), _p(y32), _stream(x))
    check(rc, "rf_add_layernorm_split_fwd")
    return yh, yl, y32


def join_split(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """fp32 values of split-stream rows (host-side torch integer ops; used on a few rows only,
    e.g. the pooled CLS rows)."""
    h = hi.view(torch.int16).to(torch.int32) & 0xFFFF
    l = lo.to(torch.int32) & 0xFFFF
    return (((h - (l >> 15)) << 16) | l).view(torch.float32)


def gemm(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
         epilogue: int = RF_EPI_BIAS, resid: Optional[torch.Tensor] = None,
         scale_cols: int = 0, col_scale: float = 1.0, out: Optional[torch.Tensor] = None,
         ra: Optional[torch.Tensor] = None, rw: Optional[torch.Tensor] = None,
         tag: Optional[str] = None, out_f32: bool = False) -> torch.Tensor:
    """C = epi(a . w^T); a (M,K), w (N,K) row-major, same dtype. out_f32 stores C in fp32."""
    lib = _lib.load()
    _dev(a, w, bias, resid)
    if a.dtype != w.dtype:
        raise TypeError(f"gemm: dtype mismatch {a.dtype} vs {w.dtype}")
    M, K = a.shape
    N, K2 = w.shape
    if K != K2:
        raise ValueError(f"gemm: K mismatch {K} vs {K2}")
    lda, ldw = _rowmajor(a, "a"), _rowmajor(w, "w")
    odt = torch.float32 if (epilogue == RF_EPI_COS or out_f32) else a.dtype
    io = 0
    if out is not None and out.dtype != odt:
        raise TypeError(f"gemm: out must be {odt}")
    if out is None:
        # 16-B aligned rows for the vector epilogue: pad the leading dim, return the (M, N) view
        n8 = (N + 7) // 8 * 8
        out = torch.empty(M, n8, dtype=odt, device=a.device)[:, :N]
    ldc = _rowmajor(out, "out")
    ldr = 0
    if resid is not None:
        ldr = _rowmajor(resid, "resid")
        if resid.dtype not in (a.dtype, torch.float32) or resid.shape != (M, N):
            raise ValueError("gemm: residual must be (M,N) in the compute dtype or fp32")
        if resid.dtype == torch.float32 and a.dtype != torch.float32:
            io |= _lib.RF_IO_R_F32
    if odt == torch.float32 and a.dtype != torch.float32 and epilogue != RF_EPI_COS:
        io |= _lib.RF_IO_C_F32
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous()):
        raise TypeError("gemm: bias must be contiguous fp32")
    with _region(tag):
        rc = lib.rf_gemm(dtype_code(a.dtype), M, N, K, _p(a), lda, _p(w), ldw, _p(bias), _p(resid),
                         ldr, _p(out), ldc, io, epilogue, scale_cols, float(col_scale), _p(ra), _p(rw),
                         _stream(out))
    check(rc, "rf_gemm")
    return out


def gemm_resid_ln(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, resid_pre: torch.Tensor,
                  mean: torch.Tensor, rstd: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                  tag: Optional[str] = None) -> torch.Tensor:
    """fp32 C = a . w^T + bias + LayerNorm(resid_pre) with the stored row stats (mean, rstd)."""
    lib = _lib.load()
    _dev(a, w, bias, resid_pre, mean, rstd)
    M, K = a.shape
    N = w.shape[0]
    if resid_pre.dtype != torch.float32 or resid_pre.shape != (M, N):
        raise ValueError("gemm_resid_ln: resid_pre must be the fp32 (M, N) pre-LayerNorm rows")
    out = torch.empty(M, N, dtype=torch.float32, device=a.device)
    with _region(tag):
        rc = lib.rf_gemm_resid_ln(dtype_code(a.dtype), M, N, K, _p(a), _rowmajor(a, "a"), _p(w),
                                  _rowmajor(w, "w"), _p(bias), _p(resid_pre),
                                  _rowmajor(resid_pre, "resid_pre"), _p(mean), _p(rstd), _p(gamma),
                                  _p(beta), _p(out), N, _stream(out))
    check(rc, "rf_gemm_resid_ln")
    return out


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float,
              out: Optional[torch.Tensor] = None, stats: bool = False, tag: Optional[str] = None,
              out_dtype: Optional[torch.dtype] = None, want_f32: bool = False):
    """y = LN(x) in out_dtype (default x.dtype); want_f32 also returns an fp32 copy.
    Returns y, or (y, y32) with want_f32, or (y, mean, rstd) with stats."""
    lib = _lib.load()
    _dev(x)
    M, D = x.shape
    ldx = _rowmajor(x, "x")
    if out is None:
        out = torch.empty(M, D, dtype=out_dtype or x.dtype, device=x.device)
    y32 = torch.empty(M, D, dtype=torch.float32, device=x.device) if want_f32 else None
    mean = rstd = None
    if stats:
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    with _region(tag):
        rc = lib.rf_layernorm_fwd(dtype_code(x.dtype), dtype_code(out.dtype), M, D, _p(x), ldx,
                                  _p(w), _p(b), float(eps), _p(out), _rowmajor(out, "out"), _p(y32),
                                  _p(mean), _p(rstd), _stream(x))
    check(rc, "rf_layernorm_fwd")
    if stats and want_f32:
        return out, y32, mean, rstd
    if stats:
        return out, mean, rstd
    if want_f32:
        return out, y32
    return out


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, w: torch.Tensor,
                  tag: Optional[str] = None):
    """rf_layernorm_bwd: (dx, dw, db) of y = LN(x) for fp32 dy (contiguous) and x (row-major)."""
    lib = _lib.load()
    _dev(dy, x, mean, rstd, w)
    M, D = x.shape
    if dy.dtype != torch.float32 or x.dtype != torch.float32:
        raise TypeError("layernorm_bwd: dy and x must be fp32")
    dy = dy.contiguous()
    wf = w.float().contiguous()
    dx = torch.empty(M, D, dtype=torch.float32, device=x.device)
    dw = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    ws = torch.empty(max(lib.rf_layernorm_bwd_workspace(M, D), 4), dtype=torch.uint8, device=x.device)
    with _region(tag):
        rc = lib.rf_layernorm_bwd(M, D, _p(dy), _p(x), _rowmajor(x, "x"), _p(mean), _p(rstd), _p(wf), _p(dx),
                                  _p(dw), _p(db), _p(ws), _stream(x))
    check(rc, "rf_layernorm_bwd")
    return dx, dw, db


def colsum(x: torch.Tensor, scale_cols: int = 0, col_scale: float = 1.0, tag: Optional[str] = None) -> torch.Tensor:
    """rf_colsum: fp32 column sums of a row-major (M, N) bf16 / fp32 matrix (bias gradients); the first
    scale_cols sums multiplied by col_scale."""
    lib = _lib.load()
    _dev(x)
    M, N = x.shape
    out = torch.empty(N, dtype=torch.float32, device=x.device)
    ws = torch.empty(max(lib.rf_colsum_workspace(M, N), 4), dtype=torch.uint8, device=x.device)
    with _region(tag):
        rc = lib.rf_colsum(dtype_code(x.dtype), M, N, _p(x), _rowmajor(x, "x"), _p(out), int(scale_cols),
                           float(col_scale), _p(ws), _stream(x))
    check(rc, "rf_colsum")
    return out


def weight_grad(dc: torch.Tensor, a: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
                scale_rows: int = 0, row_scale: float = 1.0, tag: Optional[str] = None) -> torch.Tensor:
    """rf_weight_grad: dW = dc^T a in fp32 (N, K) for 16-bit dc (M, N) and a (M, K) row-major views (the
    weight gradient of a Linear), its first scale_rows rows multiplied by row_scale; `out` given with
    accumulate=True adds into it."""
    lib = _lib.load()
    _dev(dc, a)
    M, N = dc.shape
    K = a.shape[1]
    if a.shape[0] != M or a.dtype != dc.dtype:
        raise ValueError(f"weight_grad: dc {tuple(dc.shape)} {dc.dtype} vs a {tuple(a.shape)} {a.dtype}")
    if out is None:
        if accumulate:
            raise ValueError("weight_grad: accumulate needs out")
        out = torch.empty(N, K, dtype=torch.float32, device=dc.device)
    if out.dtype != torch.float32 or tuple(out.shape) != (N, K):
        raise ValueError("weight_grad: out must be an fp32 (N, K) tensor")
    ws = torch.empty(max(lib.rf_weight_grad_workspace(M, N, K), 16), dtype=torch.uint8, device=dc.device)
    with _region(tag):
        rc = lib.rf_weight_grad(dtype_code(dc.dtype), M, N, K, _p(dc), _rowmajor(dc, "dc"), _p(a), _rowmajor(a, "a"),
                                _p(out), _rowmajor(out, "out"), int(accumulate), int(scale_rows), float(row_scale),
                                _p(ws), ws.numel(), _stream(dc))
    check(rc, "rf_weight_grad")
    return out


class WeightPack:
    """Persistent compute-dtype copies of a fixed set of fp32 weights, refreshed by ONE rf_pack_weights
    launch (the training step's weight casts and transposes). specs: dicts with src (fp32, 2-D,
    row-major), dst / dstT ((tensor, row_off) or None: the row-major copy and the transposed copy),
    scale_n / t_scale (the first scale_n source rows of the transposed copy scaled by t_scale). The
    descriptors are copied to the device once, at construction (outside any graph capture); refresh()
    only launches — it refuses sources that moved (rebuild the pack then)."""

    _DESC = None

    def __init__(self, specs, dtype: torch.dtype):
        import numpy as np
        if WeightPack._DESC is None:
            WeightPack._DESC = np.dtype([("src", "<u8"), ("dst", "<u8"), ("dstT", "<u8"), ("lda", "<i8"),
                                         ("ld_dst", "<i8"), ("ld_T", "<i8"), ("first_tile", "<i8"), ("rows", "<i4"),
                                         ("cols", "<i4"), ("row_off", "<i4"), ("scale_n", "<i4"),
                                         ("t_scale", "<f4"), ("pad", "<i4")])
            assert WeightPack._DESC.itemsize == 80
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("WeightPack: bf16 or fp16")
        self.code = dtype_code(dtype)
        self.specs = list(specs)
        d = np.zeros(len(self.specs), dtype=WeightPack._DESC)
        ntile, first = 0, []
        for i, sp in enumerate(self.specs):
            src = sp["src"]
            if src.dtype != torch.float32 or src.dim() != 2 or src.stride(1) != 1 or not src.is_cuda:
                raise ValueError("WeightPack: sources must be 2-D row-major fp32 CUDA tensors")
            rows, cols = src.shape
            dst, dstT = sp.get("dst"), sp.get("dstT")
            for t, off, width in ((dst, 0, cols), (dstT, 1, rows)):
                if t is not None:
                    buf, ro = t
                    if buf.dtype != dtype or buf.stride(1) != 1:
                        raise ValueError("WeightPack: destinations must be row-major in the compute dtype")
            d[i]["src"] = src.data_ptr()
            d[i]["lda"] = src.stride(0)
            d[i]["rows"], d[i]["cols"] = rows, cols
            ro = None
            if dst is not None:
                buf, ro = dst
                if ro + rows > buf.shape[0] or cols > buf.shape[1]:
                    raise ValueError("WeightPack: dst too small")
                d[i]["dst"], d[i]["ld_dst"] = buf.data_ptr(), buf.stride(0)
            if dstT is not None:
                buf, roT = dstT
                if ro is not None and roT != ro:
                    raise ValueError("WeightPack: dst and dstT take the same row offset")
                ro = roT
                if cols > buf.shape[0] or ro + rows > buf.shape[1]:
                    raise ValueError("WeightPack: dstT too small")
                d[i]["dstT"], d[i]["ld_T"] = buf.data_ptr(), buf.stride(0)
            d[i]["row_off"] = ro or 0
            d[i]["scale_n"] = int(sp.get("scale_n", 0))
            d[i]["t_scale"] = float(sp.get("t_scale", 1.0))
            d[i]["first_tile"] = ntile
            first.append(ntile)
            ntile += ((rows + 63) // 64) * ((cols + 63) // 64)
        table = np.repeat(np.arange(len(self.specs), dtype=np.int32),
                          [((sp["src"].shape[0] + 63) // 64) * ((sp["src"].shape[1] + 63) // 64) for sp in self.specs])
        blob = np.concatenate([d.view(np.uint8), table.view(np.uint8)])
        dev = self.specs[0]["src"].device
        self.blob = torch.from_numpy(blob).to(dev)
        self.nent, self.nblk = len(self.specs), int(table.size)
        self.ptrs = tuple(sp["src"].data_ptr() for sp in self.specs)

    def valid(self) -> bool:
        return tuple(sp["src"].data_ptr() for sp in self.specs) == self.ptrs

    def refresh(self):
        if not self.valid():
            raise RuntimeError("WeightPack: a source weight moved; build a new pack")
        base = self.blob.data_ptr()
        check(_lib.load().rf_pack_weights(self.code, base, self.nent, base + self.nent * 80, self.nblk,
                                          _stream(self.blob)), "rf_pack_weights")


def embed_ln_bwd(ids, pos, tt, ip, word, posemb, typeemb, iposemb, ln_w, eps: float, dh: torch.Tensor):
    """rf_embed_ln_bwd: (dx, dgamma, dbeta) of h = LN(Ew[ids] + Ep[pos] + Et[tt] + Ei[ip]) for the fp32
    gradient dh (M, D); tables fp32 contiguous, index streams int32 (M,)."""
    lib = _lib.load()
    _dev(ids, word, dh)
    M = ids.numel()
    D = word.shape[1]
    for t in (word, posemb, typeemb, iposemb):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.shape[1] != D:
            raise ValueError("embed_ln_bwd: tables must be contiguous fp32 of one width")
    dh = dh.float().contiguous()
    if tuple(dh.shape) != (M, D):
        raise ValueError(f"embed_ln_bwd: dh {tuple(dh.shape)} for {M} rows x {D}")
    idx = [x.reshape(-1).to(torch.int32).contiguous() for x in (ids, pos, tt, ip)]
    dx = torch.empty(M, D, dtype=torch.float32, device=dh.device)
    dw = torch.empty(D, dtype=torch.float32, device=dh.device)
    db = torch.empty_like(dw)
    ws = torch.empty(max(lib.rf_embed_ln_bwd_workspace(M, D), 16), dtype=torch.uint8, device=dh.device)
    check(lib.rf_embed_ln_bwd(M, D, *(_p(x) for x in idx), _p(word), _p(posemb), _p(typeemb), _p(iposemb),
                              _p(ln_w.float().contiguous()), float(eps), _p(dh), _p(dx), _p(dw), _p(db), _p(ws),
                              _stream(dh)), "rf_embed_ln_bwd")
    return dx, dw, db


def embedding_grad(src: torch.Tensor, index: torch.Tensor, num_rows: int, pad: Optional[int] = None) -> torch.Tensor:
    """nn.Embedding's dense weight gradient (num_rows, D) fp32 from row gradients src (M, D) and the
    token indices (M,), deterministically: a stable sort of the indices, then rf_segment_rows_sum adds
    each index's rows in token order; the padding_idx row stays zero."""
    lib = _lib.load()
    _dev(src, index)
    M, D = src.shape
    src = src.float().contiguous()
    keys, perm = torch.sort(index.reshape(-1).to(torch.int32), stable=True)
    out = torch.zeros(num_rows, D, dtype=torch.float32, device=src.device)
    ws = torch.empty(max(lib.rf_segment_rows_sum_workspace(M, D), 16), dtype=torch.uint8, device=src.device)
    check(lib.rf_segment_rows_sum(M, D, _p(src), _p(perm.to(torch.int32).contiguous()), _p(keys.contiguous()),
                                  -1 if pad is None else int(pad), _p(out), num_rows, _p(ws), _stream(src)),
          "rf_segment_rows_sum")
    return out


def drop_add_ln_fwd(t: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float, p: float,
                    seed: int, want_bf16: bool = False, mask_row_mul: int = 1):
    """rf_drop_add_ln_fwd_t: (x, y, mean, rstd) with x = dropout_p(t) + res, y = LN(x), all fp32; with
    want_bf16 also y16 = bf16(y), appended. mask_row_mul: row r draws the mask of row r * mask_row_mul
    (the CLS-only last layer's compacted rows pass Lp: the full layer's row b * Lp)."""
    lib = _lib.load()
    _dev(t, res, w, b)
    M, D = t.shape
    if t.dtype not in (torch.bfloat16, torch.float16) or res.dtype != torch.float32 or not res.is_contiguous():
        raise TypeError("drop_add_ln_fwd: t bf16 / fp16 (row-major), res contiguous fp32")
    x = torch.empty(M, D, dtype=torch.float32, device=t.device)
    y = torch.empty_like(x)
    mean = torch.empty(M, dtype=torch.float32, device=t.device)
    rstd = torch.empty_like(mean)
    y16 = torch.empty(M, D, dtype=t.dtype, device=t.device) if want_bf16 else None
    check(lib.rf_drop_add_ln_fwd_t(dtype_code(t.dtype), M, D, _p(t), _rowmajor(t, "t"), _p(res), float(p), seed,
                                   _p(w.float().contiguous()), _p(b.float().contiguous()), float(eps), _p(x),
                                   _p(y), _p(mean), _p(rstd), _p(y16), int(mask_row_mul), _stream(t)),
          "rf_drop_add_ln_fwd")
    return (x, y, mean, rstd, y16) if want_bf16 else (x, y, mean, rstd)


def drop_add_ln_bwd(dy, x, mean, rstd, w, p: float, seed: int, dy16: Optional[torch.Tensor] = None,
                    dtype: torch.dtype = torch.bfloat16, want_dbias: bool = False, mask_row_mul: int = 1):
    """rf_drop_add_ln_bwd_t: (dres fp32, dt, dw, db) for the gradient dy (fp32) of y plus, when given,
    dy16 of its 16-bit copy; either may be None (not both). dt and dy16 in `dtype` (bf16 / fp16).
    want_dbias (rf_drop_add_ln_bwd_tb): also the column sums of dt (the dense branch's bias gradient)."""
    lib = _lib.load()
    _dev(x, mean, rstd, w)
    M, D = x.shape
    if dy is None and dy16 is None:
        raise ValueError("drop_add_ln_bwd: no gradient")
    dy = None if dy is None else dy.float().contiguous()
    if dy16 is not None:
        if dy16.dtype != dtype or tuple(dy16.shape) != (M, D):
            raise TypeError(f"drop_add_ln_bwd: dy16 must be a {dtype} (M, D) tensor")
        dy16 = dy16.contiguous()
    dres = torch.empty(M, D, dtype=torch.float32, device=x.device)
    dt = torch.empty(M, D, dtype=dtype, device=x.device)
    dw = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty_like(dw)
    ws = torch.empty(max(lib.rf_layernorm_bwd_workspace(M, D), 4), dtype=torch.uint8, device=x.device)
    if want_dbias:
        dbias = torch.empty_like(dw)
        check(lib.rf_drop_add_ln_bwd_tb(dtype_code(dtype), M, D, _p(dy), _p(dy16), _p(x), _p(mean), _p(rstd),
                                        _p(w.float().contiguous()), float(p), seed, _p(dres), _p(dt), _p(dw), _p(db),
                                        _p(dbias), _p(ws), int(mask_row_mul), _stream(x)),
              "rf_drop_add_ln_bwd_tb")
        return dres, dt, dw, db, dbias
    check(lib.rf_drop_add_ln_bwd_t(dtype_code(dtype), M, D, _p(dy), _p(dy16), _p(x), _p(mean), _p(rstd),
                                   _p(w.float().contiguous()), float(p), seed, _p(dres), _p(dt), _p(dw), _p(db), _p(ws),
                                   int(mask_row_mul), _stream(x)),
          "rf_drop_add_ln_bwd")
    return dres, dt, dw, db


def scatter_add_rows(rows: torch.Tensor, src0, dst0, src1=None, dst1=None):
    """rf_scatter_add_rows: dst[rows[r]] += src[r] in place (rows int32, -1 = skip) for one or two
    (src, dst) pairs; src (R, D) and dst (*, D) row-major in one dtype (bf16 or fp32)."""
    lib = _lib.load()
    _dev(rows, src0, dst0)
    R, D = src0.shape
    pairs = [(src0, dst0)] + ([(src1, dst1)] if src1 is not None else [])
    for s_, d_ in pairs:
        if s_.dtype != d_.dtype or s_.shape != (R, D) or d_.shape[1] != D or s_.stride(0) != src0.stride(0) \
                or d_.stride(0) != dst0.stride(0):
            raise ValueError("scatter_add_rows: src/dst shapes, dtypes or strides differ")
    if rows.dtype != torch.int32 or rows.numel() != R:
        raise ValueError("scatter_add_rows: rows must be int32 with one entry per src row")
    check(lib.rf_scatter_add_rows(dtype_code(src0.dtype), R, D, _p(rows.contiguous()), _p(src0), _p(src1),
                                  _rowmajor(src0, "src"), _p(dst0), _p(dst1), _rowmajor(dst0, "dst"),
                                  _stream(dst0)), "rf_scatter_add_rows")
    return dst0, dst1


def band_attention_bwd(q, k, v, o, dout, flags, gidx, B: int, Lp: int, H: int, tag: Optional[str] = None,
                       dqkv: Optional[torch.Tensor] = None, p_drop: float = 0.0, seed: int = 0):
    """Gradient of the local branch (rf_band_attn_bwd): q/k/v (pre-scaled q) and o, dout bf16
    (B*Lp, >=H*64) views; returns (dq, dk, dv) of shape (B*Lp, H*64) — fp32, or column views of
    `dqkv` (B*Lp, 3*H*64) in its dtype (fp32 or bf16) when given — plus, when there are global keys, gds / gpr
    (B, H, Lp, gmax): dS and P of the global-key columns (P times the dropout mask / (1 - p_drop) when
    the forward ran with attention-probability dropout p_drop, seed; rf_band_attn_bwd_drop)."""
    lib = _lib.load()
    _dev(q, k, v, o, dout, flags)
    ld = _rowmajor(q, "q")
    if _rowmajor(k, "k") != ld or _rowmajor(v, "v") != ld:
        raise ValueError("band_attention_bwd: q/k/v must share a leading dimension")
    D = H * 64
    gmax = gidx.shape[1]
    dev = q.device
    if dqkv is not None:
        if (dqkv.dtype not in (torch.float32, q.dtype) or not dqkv.is_contiguous()
                or tuple(dqkv.shape) != (B * Lp, 3 * D)):
            raise ValueError("band_attention_bwd: dqkv must be a contiguous fp32 or q-dtype (B*Lp, 3*D) tensor")
        dq, dk, dv, ldg = dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:], 3 * D
    else:
        dq = torch.empty(B * Lp, D, dtype=torch.float32, device=dev)
        dk = torch.empty_like(dq)
        dv = torch.empty_like(dq)
        ldg = D
    lse2 = torch.empty(B * H * Lp, dtype=torch.float32, device=dev)
    delta = torch.empty_like(lse2)
    gds = torch.empty(B, H, Lp, max(gmax, 1), dtype=torch.float32, device=dev) if gmax else None
    gpr = torch.empty_like(gds) if gmax else None
    with _region(tag):
        rc = lib.rf_band_attn_bwd_drop(dtype_code(q.dtype), dtype_code(dq.dtype), B, Lp, H, 64, 32, _p(q), _p(k), _p(v), ld, _p(o),
                                       _rowmajor(o, "o"), _p(dout), _rowmajor(dout, "dout"), _p(flags),
                                       _p(gidx.contiguous()) if gmax else None, gmax, _p(dq), _p(dk), _p(dv), ldg,
                                       _p(lse2), _p(delta), _p(gds), _p(gpr), float(p_drop), int(seed), _stream(q))
    check(rc, "rf_band_attn_bwd")
    return dq, dk, dv, gds, gpr


def add_layernorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float,
                  out_dtype: Optional[torch.dtype] = None, res_out: Optional[torch.Tensor] = None,
                  tag: Optional[str] = None):
    """y = LN(x + res) (rf_add_layernorm_fwd): x the dense output (bf16 under autocast, as the
    reference's Linear returns it), res the fp32 residual stream (M, D) contiguous. Returns
    (y in out_dtype, y32 fp32); y32 is `res_out` when given, which may be `res` itself (the
    stream updated in place)."""
    lib = _lib.load()
    _dev(x, res)
    M, D = x.shape
    if res.dtype != torch.float32 or not res.is_contiguous() or tuple(res.shape) != (M, D):
        raise ValueError("add_layernorm: res must be a contiguous fp32 (M, D) tensor")
    y = torch.empty(M, D, dtype=out_dtype or x.dtype, device=x.device)
    y32 = res_out if res_out is not None else torch.empty(M, D, dtype=torch.float32, device=x.device)
    if y32.dtype != torch.float32 or not y32.is_contiguous() or tuple(y32.shape) != (M, D):
        raise ValueError("add_layernorm: res_out must be a contiguous fp32 (M, D) tensor")
    with _region(tag):
        rc = lib.rf_add_layernorm_fwd(dtype_code(x.dtype), dtype_code(y.dtype), M, D, _p(x), _rowmajor(x, "x"),
                                      _p(res), _p(w), _p(b), float(eps), _p(y), _rowmajor(y, "y"), _p(y32),
                                      None, None, _stream(x))
    check(rc, "rf_add_layernorm_fwd")
    return y, y32


def band_attention(q, k, v, flags, gidx, B: int, Lp: int, H: int, half_w: int,
                   out: Optional[torch.Tensor] = None, tag: Optional[str] = None, p_drop: float = 0.0,
                   seed: int = 0):
    """q/k/v: (B*Lp, >=H*64) row-major views sharing one leading dim (e.g. column slices of
    the fused projection output). p_drop > 0: attention-probability dropout (training, TF:585-586)
    with the counter-hash mask of `seed` (rf_band_attn_fwd_drop)."""
    lib = _lib.load()
    _dev(q, k, v, flags)
    ld = _rowmajor(q, "q")
    if _rowmajor(k, "k") != ld or _rowmajor(v, "v") != ld:
        raise ValueError("band_attention: q/k/v must share a leading dimension")
    D = H * 64
    if out is None:
        out = torch.empty(B * Lp, D, dtype=q.dtype, device=q.device)
    gmax = gidx.shape[1]
    with _region(tag):
        rc = lib.rf_band_attn_fwd_drop(dtype_code(q.dtype), B, Lp, H, 64, half_w, _p(q), _p(k), _p(v), ld,
                                       _p(flags), _p(gidx) if gmax else None, gmax, _p(out),
                                       _rowmajor(out, "out"), float(p_drop), int(seed), _stream(out))
    check(rc, "rf_band_attn_fwd")
    return out


def global_attention(qg, kg, vg, flags, gidx, B: int, Lp: int, H: int, out: torch.Tensor,
                     tag: Optional[str] = None):
    lib = _lib.load()
    gmax = gidx.shape[1]
    if gmax == 0:
        return out
    ld = _rowmajor(kg, "kg")
    if _rowmajor(vg, "vg") != ld:
        raise ValueError("global_attention: kg/vg must share a leading dimension")
    with _region(tag):
        rc = lib.rf_global_attn_fwd(dtype_code(qg.dtype), B, Lp, H, 64, _p(qg), _rowmajor(qg, "qg"),
                                    _p(kg), _p(vg), ld, _p(flags), _p(gidx.contiguous()), gmax,
                                    _p(out), _rowmajor(out, "out"), _stream(out))
    check(rc, "rf_global_attn_fwd")
    return out


def global_attention_fold(qg, h, wkg, bkg, wvg, bvg, flags, gidx, B: int, Lp: int, H: int,
                          out: Optional[torch.Tensor], tag: Optional[str] = None, p_drop: float = 0.0, seed: int = 0,
                          ws: Optional[torch.Tensor] = None, stage: int = 3):
    """Global query rows through the key/value-projection fold (rf_global_attn_fold_fwd_drop):
    overwrites ctx rows at the global positions; p_drop > 0: attention-probability dropout with
    the counter-hash mask of `seed` (16-bit dtypes). ws: the fold workspace to use (a training
    forward keeps it for global_fold_bwd), else a fresh one. stage 1 / 2 (rf_global_attn_fold_fwd_stage):
    the pass over h only (out unused, may be None) / the merge and output only, on the same ws."""
    lib = _lib.load()
    gmax = gidx.shape[1]
    if gmax == 0:
        return out
    _dev(qg, h, wkg, wvg, flags)
    D = h.shape[1]
    ws_bytes = lib.rf_global_fold_workspace(B, Lp, D, H, gmax)
    if ws is None:
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=h.device)
    elif ws.numel() < ws_bytes:
        raise ValueError("global_attention_fold: workspace too small")
    for t in (wkg, wvg):
        if not t.is_contiguous() or t.dtype != h.dtype:
            raise ValueError("global_attention_fold: weights must be contiguous in the compute dtype")
    if stage not in (1, 2, 3) or (out is None and stage != 1):
        raise ValueError(f"global_attention_fold: stage {stage} with out {'None' if out is None else 'given'}")
    ldo = _rowmajor(out, "out") if out is not None else D
    with _region(tag):
        rc = lib.rf_global_attn_fold_fwd_stage(stage, dtype_code(h.dtype), B, Lp, D, H, _p(qg), _rowmajor(qg, "qg"),
                                               _p(h), _rowmajor(h, "h"), _p(wkg), _p(bkg), _p(wvg), _p(bvg),
                                               _p(flags), _p(gidx.contiguous()), gmax, _p(ws), _p(out), ldo,
                                               float(p_drop), int(seed) & (2**64 - 1), _stream(h))
    check(rc, "rf_global_attn_fold_fwd_stage")
    return out


def global_fold_bwd(h, flags, gidx, B: int, Lp: int, H: int, fwd_ws: torch.Tensor, dw: torch.Tensor,
                    cb: Optional[torch.Tensor], p_drop: float, seed: int, dh: torch.Tensor):
    """rf_global_fold_bwd: the global rows' backward in one pass over h from the forward's fold
    workspace. dw (R, 16, D) fp32, cb (R, 16) fp32 or None; writes dh (B*Lp, D) in h's dtype and
    returns (du, w, stats): (R, 16, D), (R, 16, D) fp32 and (R, 16, 4) fp32 (M, 1/L, Delta, S')."""
    lib = _lib.load()
    gmax = gidx.shape[1]
    D = h.shape[1]
    R = B * gmax
    dev = h.device
    if tuple(dw.shape) != (R, 16, D) or dw.dtype != torch.float32 or not dw.is_contiguous():
        raise ValueError("global_fold_bwd: dw must be contiguous fp32 (R, 16, D)")
    if cb is not None and (tuple(cb.shape) != (R, 16) or cb.dtype != torch.float32 or not cb.is_contiguous()):
        raise ValueError("global_fold_bwd: cb must be contiguous fp32 (R, 16)")
    du = torch.empty(R, 16, D, dtype=torch.float32, device=dev)
    w = torch.empty_like(du)
    stats = torch.empty(R, 16, 4, dtype=torch.float32, device=dev)
    ws = torch.empty(max(lib.rf_global_fold_bwd_workspace(B, Lp, D, gmax), 16), dtype=torch.uint8, device=dev)
    check(lib.rf_global_fold_bwd(dtype_code(h.dtype), B, Lp, D, H, _p(h), _rowmajor(h, "h"), _p(flags),
                                 _p(gidx.to(torch.int32).contiguous()), gmax, _p(fwd_ws), _p(dw), _p(cb),
                                 float(p_drop), int(seed) & (2**64 - 1), _p(dh), _rowmajor(dh, "dh"), _p(du), _p(w),
                                 _p(stats), _p(ws), _stream(h)), "rf_global_fold_bwd")
    return du, w, stats


def global_fold_bwd_full(h, flags, gidx, B: int, Lp: int, H: int, fwd_ws: torch.Tensor, dout, qg, wkg, wvg, bvg,
                         p_drop: float, seed: int, dh: torch.Tensor, want_dbkg: bool = True):
    """rf_global_fold_bwd_full: the global branch's whole backward from the attention output gradient
    dout (B*Lp, >= D) 16-bit: writes dh (B*Lp, D) in h's dtype and returns fp32 (dqg (R, D), dwkg
    (D, D), dbkg (D) of zeros or None, dwvg (D, D), dbvg (D)). qg (R, D) the forward's scaled
    query_global rows; wkg / wvg (D, D) and bvg (D,) the weights the forward used."""
    lib = _lib.load()
    gmax = gidx.shape[1]
    D = h.shape[1]
    R = B * gmax
    dev = h.device
    for name, t in (("qg", qg), ("wkg", wkg), ("wvg", wvg)):
        if t.dtype != h.dtype or t.stride(-1) != 1:
            raise ValueError(f"global_fold_bwd_full: {name} must be row-major in h's dtype")
    if tuple(wkg.shape) != (D, D) or tuple(wvg.shape) != (D, D) or not wkg.is_contiguous() or not wvg.is_contiguous():
        raise ValueError("global_fold_bwd_full: wkg / wvg must be contiguous (D, D)")
    bvg = bvg.float().contiguous()
    dqg = torch.empty(R, D, dtype=torch.float32, device=dev)
    dwkg = torch.empty(D, D, dtype=torch.float32, device=dev)
    dwvg = torch.empty_like(dwkg)
    dbvg = torch.empty(D, dtype=torch.float32, device=dev)
    dbkg = torch.empty(D, dtype=torch.float32, device=dev) if want_dbkg else None
    ws = torch.empty(max(lib.rf_global_fold_bwd_full_workspace(B, Lp, D, gmax), 16), dtype=torch.uint8, device=dev)
    check(lib.rf_global_fold_bwd_full(dtype_code(h.dtype), B, Lp, D, H, _p(h), _rowmajor(h, "h"), _p(flags),
                                      _p(gidx.to(torch.int32).contiguous()), gmax, _p(fwd_ws), _p(dout),
                                      _rowmajor(dout, "dout"), _p(qg), _rowmajor(qg, "qg"), _p(wkg), _p(wvg), _p(bvg),
                                      float(p_drop), int(seed) & (2**64 - 1), _p(dh), _rowmajor(dh, "dh"), _p(dqg),
                                      _p(dwkg), _p(dwvg), _p(dbvg), _p(dbkg), _p(ws), _stream(h)),
          "rf_global_fold_bwd_full")
    return dqg, dwkg, dbkg, dwvg, dbvg


def global_kv_grad(gds, gpr, q, dout, gidx, B: int, Lp: int, H: int, dk, dv):
    """rf_global_kv_grad: dk / dv (16-bit row-major views, e.g. column slices of the fused dqkv) +=
    the global-key / global-value rows' gradients reduced from the band backward's (B, H, Lp, gmax)
    fp32 gds / gpr against q / dout (16-bit), at the global positions gidx (in place)."""
    gmax = gidx.shape[1]
    for name, t in (("gds", gds), ("gpr", gpr)):
        if tuple(t.shape) != (B, H, Lp, gmax) or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"global_kv_grad: {name} must be contiguous fp32 (B, H, Lp, gmax)")
    for name, t in (("dout", dout), ("dk", dk), ("dv", dv)):
        if t.dtype != q.dtype:
            raise ValueError(f"global_kv_grad: {name} must have q's dtype")
    check(_lib.load().rf_global_kv_grad(dtype_code(q.dtype), B, Lp, H, gmax, _p(gds), _p(gpr), _p(q),
                                        _rowmajor(q, "q"), _p(dout), _rowmajor(dout, "dout"),
                                        _p(gidx.to(torch.int32).contiguous()), _p(dk), _rowmajor(dk, "dk"), _p(dv),
                                        _rowmajor(dv, "dv"), _stream(q)), "rf_global_kv_grad")


def global_query_bwd(gidx, dqg, q_scale: float, h, wqgT, dh, B: int, Lp: int):
    """rf_global_query_bwd: backward of qg = (h[global rows] Wqg^T + bqg) * q_scale from dqg (R, D)
    fp32: returns fp32 (dWqg (D, D), dbqg (D,)) and adds the global rows' input gradient into dh (in
    place). wqgT (D, D): Wqg^T * q_scale in h's dtype."""
    gmax = gidx.shape[1]
    D = h.shape[1]
    if tuple(dqg.shape) != (B * gmax, D) or dqg.dtype != torch.float32 or not dqg.is_contiguous():
        raise ValueError("global_query_bwd: dqg must be contiguous fp32 (B*gmax, D)")
    if tuple(wqgT.shape) != (D, D) or wqgT.dtype != h.dtype or not wqgT.is_contiguous() or dh.dtype != h.dtype:
        raise ValueError("global_query_bwd: wqgT (D, D) contiguous and dh in h's dtype")
    dwqg = torch.empty(D, D, dtype=torch.float32, device=h.device)
    dbqg = torch.empty(D, dtype=torch.float32, device=h.device)
    check(_lib.load().rf_global_query_bwd(dtype_code(h.dtype), B, Lp, D, gmax, _p(gidx.to(torch.int32).contiguous()),
                                          _p(dqg), float(q_scale), _p(h), _rowmajor(h, "h"), _p(wqgT), _p(dwqg),
                                          _p(dbqg), _p(dh), _rowmajor(dh, "dh"), _stream(h)), "rf_global_query_bwd")
    return dwqg, dbqg


def attn_global_keep(gidx, B: int, Lp: int, H: int, p_drop: float, seed: int) -> torch.Tensor:
    """(B, H, gmax, Lp) fp32 attention-dropout scale of the global query rows (rf_attn_global_keep;
    the mask rf_global_attn_fold_fwd_drop applies)."""
    gmax = gidx.shape[1]
    z = torch.empty(B, H, gmax, Lp, dtype=torch.float32, device=gidx.device)
    g32 = gidx.to(torch.int32).contiguous()
    rc = _lib.load().rf_attn_global_keep(B, H, Lp, _p(g32), gmax, float(p_drop), int(seed) & (2**64 - 1), _p(z),
                                         _stream(z))
    check(rc, "rf_attn_global_keep")
    return z


def global_attention_fold_h(h, wqg, bqg, q_scale: float, wkg, bkg, wvg, bvg, flags, gidx, B: int, Lp: int,
                            H: int, out: torch.Tensor, tag: Optional[str] = None):
    """Whole global path of a layer from its input h (rf_global_attn_fold_h_fwd): query_global
    projection of the global rows, then the key/value-projection fold; overwrites ctx rows at
    the global positions."""
    lib = _lib.load()
    gmax = gidx.shape[1]
    if gmax == 0:
        return out
    _dev(h, wqg, wkg, wvg, flags)
    D = h.shape[1]
    for t in (wqg, wkg, wvg):
        if not t.is_contiguous() or t.dtype != h.dtype:
            raise ValueError("global_attention_fold_h: weights must be contiguous in the compute dtype")
    ws_bytes = lib.rf_global_fold_workspace(B, Lp, D, H, gmax)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=h.device)
    with _region(tag):
        rc = lib.rf_global_attn_fold_h_fwd(dtype_code(h.dtype), B, Lp, D, H, _p(h), _rowmajor(h, "h"), _p(wqg),
                                           _p(bqg), float(q_scale), _p(wkg), _p(bkg), _p(wvg), _p(bvg),
                                           _p(flags), _p(gidx.contiguous()), gmax, _p(ws), _p(out),
                                           _rowmajor(out, "out"), _stream(out))
    check(rc, "rf_global_attn_fold_h_fwd")
    return out


def global_fold_workspace(h, B: int, Lp: int, H: int, gmax: int) -> torch.Tensor:
    ws_bytes = _lib.load().rf_global_fold_workspace(B, Lp, h.shape[1], H, gmax)
    return torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=h.device)


def global_attention_fold_h_stage(stage: int, ws: torch.Tensor, h, wqg, bqg, q_scale: float, wkg, bkg, wvg, bvg,
                                  flags, gidx, B: int, Lp: int, H: int, out: Optional[torch.Tensor] = None,
                                  tag: Optional[str] = None):
    """rf_global_attn_fold_h_stage: stage 1 (query_global projection + partial softmax over h,
    into `ws`), stage 2 (merge + value fold from `ws` into the global rows of `out`)."""
    lib = _lib.load()
    gmax = gidx.shape[1]
    if gmax == 0:
        return out
    if stage & 2 and out is None:
        raise ValueError("global_attention_fold_h_stage: stage 2 writes `out`")
    _dev(h, wqg, wkg, wvg, flags, ws)
    D = h.shape[1]
    for t in (wqg, wkg, wvg):
        if not t.is_contiguous() or t.dtype != h.dtype:
            raise ValueError("global_attention_fold_h_stage: weights must be contiguous in the compute dtype")
    if ws.numel() < lib.rf_global_fold_workspace(B, Lp, D, H, gmax):
        raise ValueError("global_attention_fold_h_stage: workspace too small")
    with _region(tag):
        rc = lib.rf_global_attn_fold_h_stage(int(stage), dtype_code(h.dtype), B, Lp, D, H, _p(h), _rowmajor(h, "h"),
                                             _p(wqg), _p(bqg), float(q_scale), _p(wkg), _p(bkg), _p(wvg), _p(bvg),
                                             _p(flags), _p(gidx.contiguous()), gmax, _p(ws), _p(out),
                                             D if out is None else _rowmajor(out, "out"), _stream(h))
    check(rc, "rf_global_attn_fold_h_stage")
    return out


def gather_global_rows(x, gidx, B: int, Lp: int):
    lib = _lib.load()
    gmax = gidx.shape[1]
    D = x.shape[1]
    out = torch.empty(B * gmax, D, dtype=x.dtype, device=x.device)
    check(lib.rf_gather_global_rows(dtype_code(x.dtype), B, Lp, D, gmax, _p(x), _rowmajor(x, "x"),
                                    _p(gidx.contiguous()), _p(out), _stream(out)),
          "rf_gather_global_rows")
    return out


def row_inv_norm(x: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    lib = _lib.load()
    _dev(x)
    M, D = x.shape
    out = torch.empty(M, dtype=torch.float32, device=x.device)
    check(lib.rf_row_inv_norm(dtype_code(x.dtype), M, D, _p(x), _rowmajor(x, "x"), float(eps),
                              _p(out), _stream(x)), "rf_row_inv_norm")
    return out


def cos_scores(z: torch.Tensor, items: torch.Tensor, inv_temp: float,
               z_rnorm: Optional[torch.Tensor] = None,
               items_rnorm: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B,N) fp32 = cos(z_b, items_n) * inv_temp on the MFMA GEMM (Similarity, models.py:358-369)."""
    if z_rnorm is None:
        z_rnorm = row_inv_norm(z)
    if items_rnorm is None:
        items_rnorm = row_inv_norm(items)
    return gemm(z, items, None, RF_EPI_COS, col_scale=inv_temp, ra=z_rnorm, rw=items_rnorm, out=out)


def cos_scores_cand(z: torch.Tensor, items: torch.Tensor, cand: torch.Tensor, inv_temp: float,
                    z_rnorm: Optional[torch.Tensor] = None,
                    items_rnorm: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = _lib.load()
    _dev(z, items, cand)
    B, D = z.shape
    C = cand.shape[1]
    if z_rnorm is None:
        z_rnorm = row_inv_norm(z)
    if items_rnorm is None:
        items_rnorm = row_inv_norm(items)
    cand = cand.to(torch.int64).contiguous()
    out = torch.empty(B, C, dtype=torch.float32, device=z.device)
    check(lib.rf_cos_score_cand(dtype_code(z.dtype), B, C, D, _p(z), _rowmajor(z, "z"), _p(z_rnorm),
                                _p(items), _rowmajor(items, "items"), _p(items_rnorm), _p(cand),
                                float(inv_temp), _p(out), _stream(out)), "rf_cos_score_cand")
    return out


def cos_scores_bwd(z: torch.Tensor, items: torch.Tensor, g: torch.Tensor, s: torch.Tensor, inv_temp: float,
                   z_rnorm: torch.Tensor, items_rnorm: torch.Tensor,
                   cand: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rf_cos_score_bwd: dL/dz (B, D) fp32 of the cosine scores s = cos(z_b, items_n) * inv_temp
    (n = column, or cand[b, c] for sampled candidates) from their gradient g (B, C) fp32 and s
    itself; z_rnorm / items_rnorm are the forward's inverse norms (Similarity's backward,
    models.py:358-369 under the CrossEntropyLoss of :583-599)."""
    lib = _lib.load()
    _dev(z, items, g, s, z_rnorm, items_rnorm)
    B, D = z.shape
    C = g.shape[1]
    if items.dtype != z.dtype:
        raise TypeError(f"cos_scores_bwd: items {items.dtype} vs z {z.dtype}")
    for t, nm in ((g, "g"), (s, "s")):
        if t.dtype != torch.float32 or tuple(t.shape) != (B, C):
            raise ValueError(f"cos_scores_bwd: {nm} must be fp32 ({B}, {C})")
    if cand is not None:
        cand = cand.to(torch.int64).contiguous()
        if tuple(cand.shape) != (B, C):
            raise ValueError("cos_scores_bwd: cand must be (B, C)")
    elif C > items.shape[0]:
        raise ValueError("cos_scores_bwd: more score columns than items")
    ws = torch.empty(max(int(lib.rf_cos_score_bwd_workspace(B, C, D)), 4), dtype=torch.uint8, device=z.device)
    dz = torch.empty(B, D, dtype=torch.float32, device=z.device)
    check(lib.rf_cos_score_bwd(dtype_code(z.dtype), B, C, D, _p(z), _rowmajor(z, "z"), _p(z_rnorm.contiguous()),
                               _p(items), _rowmajor(items, "items"), _p(items_rnorm.contiguous()), _p(cand),
                               float(inv_temp), _p(g), _rowmajor(g, "g"), _p(s), _rowmajor(s, "s"), _p(ws), _p(dz),
                               D, _stream(dz)), "rf_cos_score_bwd")
    return dz


def cross_entropy_bwd(logits: torch.Tensor, labels: torch.Tensor, grad_scale: torch.Tensor,
                      ignore_index: int = -100) -> torch.Tensor:
    """rf_cross_entropy_bwd: d(mean CE)/d(logits) = (softmax - onehot) * grad_scale (a one-element
    fp32 device tensor: upstream gradient / counted rows), zero rows for ignore_index; same dtype
    and shape as logits."""
    lib = _lib.load()
    _dev(logits, labels, grad_scale)
    M, N = logits.shape
    labels = labels.reshape(-1).to(torch.int64).contiguous()
    if labels.numel() != M:
        raise ValueError(f"cross_entropy_bwd: {labels.numel()} labels for {M} rows")
    gs = grad_scale.reshape(-1).to(torch.float32).contiguous()
    out = torch.empty(M, N, dtype=logits.dtype, device=logits.device)
    check(lib.rf_cross_entropy_bwd(dtype_code(logits.dtype), M, N, _p(logits), _rowmajor(logits, "logits"),
                                   _p(labels), int(ignore_index), _p(gs), _p(out), N, _stream(out)),
          "rf_cross_entropy_bwd")
    return out


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100,
                  reduction: str = "mean", want_argmax: bool = False):
    """torch.nn.functional.cross_entropy over rows of a (M, N) fp32/bf16 logits view, in fp32 on
    the HIP kernel (rf_cross_entropy_fwd); mean over the non-ignored rows (nan if none, as torch).
    want_argmax also returns the int64 row argmax (models.py:497)."""
    lib = _lib.load()
    _dev(logits, labels)
    M, N = logits.shape
    labels = labels.reshape(-1).to(torch.int64).contiguous()
    if labels.numel() != M:
        raise ValueError(f"cross_entropy: {labels.numel()} labels for {M} rows")
    rows = torch.empty(M, dtype=torch.float32, device=logits.device)
    amax = torch.empty(M, dtype=torch.int32, device=logits.device) if want_argmax else None
    check(lib.rf_cross_entropy_fwd(dtype_code(logits.dtype), M, N, _p(logits), _rowmajor(logits, "logits"),
                                   _p(labels), int(ignore_index), _p(rows), _p(amax), _stream(rows)),
          "rf_cross_entropy_fwd")
    if reduction == "none":
        loss = rows
    elif reduction == "sum":
        loss = rows.sum()
    else:
        loss = rows.sum() / (labels != ignore_index).sum().to(torch.float32)
    if want_argmax:
        return loss, amax.to(torch.int64)
    return loss
