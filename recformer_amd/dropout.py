"""Dropout keep masks of the training path as torch tensor ops.

The HIP kernels draw dropout masks from a counter hash of (seed, element index) and regenerate
them in the backward instead of storing them (rf_common.h `drop_keep`). This module states the
same hash bit-exactly with int64 torch ops (32-bit products split into 16-bit halves, so nothing
overflows), for the parts of the training path that run as torch ops on the device: the global
query rows under attention-probability dropout (TF:1036-1037) and the fp32 recompute of the
attention (TF:585-586).

Attention-probability dropout index: ((b*H + h)*Lp + i)*Lp + j for sequence b, head h, query
position i and key position j (padded length Lp); keep iff hash >= thresh, kept values scaled by
1 / (1 - p), as nn.functional.dropout.
"""
from __future__ import annotations

import numpy as np
import torch

_M32 = 0xFFFFFFFF
_MIX = 0x9E3779B97F4A7C15  # SEED_STEP_MIX of rf_common.h
_seed_counter = None  # device int64 step counter of a captured step (set_seed_counter), or None


def set_seed_counter(counter):
    """Mirror of rf_set_seed_source for the torch-side masks: while a device step counter is set,
    the seed of every mask drawn here is seed + counter * SEED_STEP_MIX (mod 2^64), computed on the
    device, exactly as the kernels resolve theirs — so a captured step's torch-side dropout (the
    non-fold global rows, the fp32 recompute) also draws fresh masks on each replay. Returns the
    previous counter."""
    global _seed_counter
    old, _seed_counter = _seed_counter, counter
    return old


def _signed64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def drop_params(p: float):
    """(thresh, scale) exactly as the kernels compute them from a float p: thresh =
    uint32(double(float(p)) * 2^32), scale = 1.0f / (1.0f - p) in fp32."""
    pf = np.float32(p)
    if pf <= 0:
        return 0, 1.0
    thresh = 0xFFFFFFFF if pf >= 1 else int(float(pf) * 4294967296.0)
    scale = float(np.float32(1.0) / (np.float32(1.0) - pf))
    return thresh, scale


def _mul32(a: torch.Tensor, c: int) -> torch.Tensor:
    """(a * c) mod 2^32 for int64 a in [0, 2^32) and a 32-bit constant c, without overflow."""
    lo = a & 0xFFFF
    hi = a >> 16
    return (lo * c + (((hi * c) & 0xFFFF) << 16)) & _M32


def keep(seed: int, idx: torch.Tensor, thresh: int) -> torch.Tensor:
    """drop_keep(seed, idx, thresh) of rf_common.h for an int64 index tensor (idx >= 0)."""
    idx = idx.to(torch.int64)
    if _seed_counter is not None:
        # seed + counter * MIX in wrapping int64 (= the kernels' uint64 arithmetic), on the device
        sd = _seed_counter.to(device=idx.device, dtype=torch.int64).reshape(()) * _signed64(_MIX) + _signed64(seed)
        s_lo, s_hi = sd & _M32, (sd >> 32) & _M32
    else:
        s_lo, s_hi = seed & _M32, (seed >> 32) & _M32
    h = _mul32(idx & _M32, 0x9E3779B1) ^ _mul32((idx >> 32) & _M32, 0x85EBCA77) ^ s_lo
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ s_hi
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    h = h ^ (h >> 16)
    return h >= thresh


def attn_scale(seed: int, p: float, row: torch.Tensor, key: torch.Tensor, Lp: int) -> torch.Tensor:
    """Keep mask x 1/(1-p) (fp32) for attention entries with mask row index row = (b*H + h)*Lp + i
    and key position key (broadcast together); invalid keys (< 0) get 0."""
    thresh, scale = drop_params(p)
    if thresh == 0:
        return torch.ones(torch.broadcast_shapes(row.shape, key.shape), dtype=torch.float32, device=row.device)
    k = key.to(torch.int64)
    kp = keep(seed, row.to(torch.int64) * Lp + k.clamp(min=0), thresh) & (k >= 0)
    return kp.to(torch.float32) * scale
