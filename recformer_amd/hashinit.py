"""Portable, bit-reproducible synthetic weights for a Recformer state dict.

Every parameter element is a pure function of (parameter name, element index):
a 32-bit integer hash (murmur3 finaliser) mapped to a uniform value. Because it
is integer arithmetic in numpy, the GPU box regenerates exactly the bytes the
golden fixtures were made with in the build container, so fixtures store seeds
and outputs, never 148M parameters (SURVEY.md §8c "portable integer-hash
weight generator").

Scale follows the reference initialiser (`LongformerPreTrainedModel._init_weights`,
N(0, initializer_range=0.02)): linear/embedding weights are uniform with std 0.02,
biases are small, LayerNorm weight is 1 + small and bias small so that the LN
affine parameters are exercised by the parity tests.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch

_U32 = np.uint32


def _mix32(x: np.ndarray) -> np.ndarray:
    """murmur3 fmix32 on uint32 arrays (wrapping arithmetic)."""
    x = x.astype(_U32, copy=True)
    x ^= x >> _U32(16)
    x *= _U32(0x85EBCA6B)
    x ^= x >> _U32(13)
    x *= _U32(0xC2B2AE35)
    x ^= x >> _U32(16)
    return x


def hash_uniform(name: str, n: int, seed: int = 0) -> np.ndarray:
    """n values uniform in [-1, 1), float64, deterministic in (seed, name, index)."""
    key = (zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        lo = (idx & np.uint64(0xFFFFFFFF)).astype(_U32)
        hi = (idx >> np.uint64(32)).astype(_U32)
        h = _mix32(lo ^ _U32(key))
        h = _mix32(h ^ (hi * _U32(0x27D4EB2F)) ^ _U32((key * 0x165667B1) & 0xFFFFFFFF))
    # 24 high bits -> [0,1) exactly representable in fp32
    u = (h >> _U32(8)).astype(np.float64) * (1.0 / (1 << 24))
    return u * 2.0 - 1.0


_SQRT3 = 3.0 ** 0.5


def hash_tensor(name: str, shape, kind: str, seed: int = 0, std: float = 0.02) -> torch.Tensor:
    n = int(np.prod(shape)) if len(shape) else 1
    u = hash_uniform(name, n, seed)
    if kind == "weight":
        v = u * (std * _SQRT3)
    elif kind == "bias":
        v = u * 0.02
    elif kind == "ln_weight":
        v = 1.0 + u * 0.1
    elif kind == "ln_bias":
        v = u * 0.05
    else:
        raise ValueError(kind)
    return torch.from_numpy(v.astype(np.float32).reshape(shape))


def _kind_for(name: str) -> str:
    leaf = name.rsplit(".", 2)
    is_ln = "LayerNorm" in name or "layer_norm" in name
    if name.endswith(".bias"):
        return "ln_bias" if is_ln else "bias"
    if is_ln:
        return "ln_weight"
    return "weight"


@torch.no_grad()
def hash_init_(module: torch.nn.Module, seed: int = 0, std: float = 0.02) -> torch.nn.Module:
    """Overwrite every floating parameter of `module` in place with hashed values.

    Embedding rows at `padding_idx` are zeroed, as nn.Embedding(padding_idx=...)
    does at construction (reference models.py:89, :104-106).
    """
    for name, p in module.named_parameters():
        if not p.is_floating_point():
            continue
        t = hash_tensor(name, tuple(p.shape), _kind_for(name), seed, std)
        p.copy_(t.to(p.dtype))
    for mname, m in module.named_modules():
        if isinstance(m, torch.nn.Embedding) and m.padding_idx is not None:
            m.weight[m.padding_idx].zero_()
    return module
