"""HIP-graph replay of inference forwards (small serving batches).

An inference forward of `RecformerModel` / `RecformerForSeqRec` is ~150 kernel launches, each
preceded by Python argument checks and a ctypes call; at a few sequences per batch the host side,
not the GPU, sets the latency. `GraphedForward` captures one forward for a fixed batch shape into
a HIP graph (torch.cuda.CUDAGraph, i.e. hipGraph on ROCm) and replays it: new inputs are copied
into the captured input buffers, one graph launch runs every kernel, and the outputs are the
captured output tensors (overwritten by each replay).

The library itself never allocates, synchronises or reads back inside a forward except for one
host read of the number of global tokens per sequence (models.RecformerModel._encode); during
capture that count is fixed to the example batch's (models._STATIC_GMAX). A replay batch with
more global tokens per sequence than the example is rejected (check=True reads the count back:
one host read instead of ~150 launches), and attention_mask / global_attention_mask keep their
meaning otherwise (ragged lengths and fewer globals are fine: the masks are inputs of the graph).
"""
from __future__ import annotations

from typing import Dict

import torch

from . import models


class GraphedForward:
    """Capture `module(**example)` (inference, no grad) once; `__call__(**batch)` replays it.

        g = GraphedForward(model, example_batch)   # example tensors on the GPU, fixed shapes
        scores = g(**batch)                        # same keys / shapes / dtypes as the example
    """

    def __init__(self, module: torch.nn.Module, example: Dict[str, torch.Tensor], warmup: int = 2,
                 check: bool = True):
        if not all(isinstance(v, torch.Tensor) and v.is_cuda for v in example.values()):
            raise ValueError("GraphedForward: example inputs must be tensors on the GPU")
        self.module = module
        self.check = check
        self.static = {k: v.clone() for k, v in example.items()}
        self.gmax = self._global_count(self.static)
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        old = models._STATIC_GMAX
        try:
            models._STATIC_GMAX = self.gmax
            with torch.no_grad():
                with torch.cuda.stream(stream):  # warm-up: caches, packed weights, kernel attributes
                    for _ in range(max(1, warmup)):
                        module(**self.static)
                torch.cuda.current_stream().wait_stream(stream)
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph):
                    self.out = module(**self.static)
        finally:
            models._STATIC_GMAX = old

    @staticmethod
    def _global_count(b: Dict[str, torch.Tensor]) -> int:
        gam = b.get("global_attention_mask")
        if gam is None:
            return 0
        gm = gam != 0
        am = b.get("attention_mask")
        if am is not None:
            gm = gm & (am > 0)
        return int(gm.sum(1).max().item()) if gm.shape[0] > 0 else 0

    def __call__(self, **batch):
        if batch.keys() != self.static.keys():
            raise ValueError(f"GraphedForward: inputs {sorted(batch)} != captured {sorted(self.static)}")
        for k, v in batch.items():
            if v.shape != self.static[k].shape or v.dtype != self.static[k].dtype:
                raise ValueError(f"GraphedForward: {k} {tuple(v.shape)} {v.dtype} != captured "
                                 f"{tuple(self.static[k].shape)} {self.static[k].dtype}")
            self.static[k].copy_(v, non_blocking=True)
        if self.check and self._global_count(self.static) > self.gmax:
            raise ValueError(f"GraphedForward: more global tokens per sequence than captured ({self.gmax})")
        self.graph.replay()
        return self.out
