"""AdamW with the whole step as one HIP launch (rf_adamw_step).

The reference trains every model with torch.optim.AdamW (optimization.py:28-32 for finetuning,
litmodels.py:42-56 for pretraining, stepped through GradScaler in fp16 runs, finetune.py:116-126).
`AdamW` here is a drop-in: the same constructor, parameter groups, state_dict layout
({'step', 'exp_avg', 'exp_avg_sq'} per parameter) and update rule as torch's non-capturable AdamW
(amsgrad=False), with the update of every tensor fused into a single pass over
(param, grad, exp_avg, exp_avg_sq) — 28 bytes of HBM traffic per fp32 element instead of
torch's multi-tensor sequence of ~8 passes. Step counts and bias corrections stay on the host as
in torch.

capturable=True (as torch's flag): the step counts live on the device, are advanced by a
foreach add and the bias corrections are computed in the kernel, so a whole training step including
the optimizer can be captured in a HIP graph (recformer_amd.graphs). Each group's learning rate and
decay factor (1 - lr * weight_decay) live in a device tensor that the kernel reads and that the host
refreshes outside the graph (`sync_hyper()`, called by every uncaptured step and by
CapturedTrainStep before each replay): an LR scheduler stepped on the host between replays
(optimization.py:7-19's linear warmup/decay, litmodels.py:57-62) reaches the captured update, as
torch's capturable AdamW with a Tensor lr. betas / eps / weight_decay changes after capture need a
re-capture (the descriptors keep them).

GradScaler (torch.amp): the optimizer sets `_step_supports_amp_scaling`, so `scaler.step(opt)` hands
it the scaler's device `grad_scale` and `found_inf` instead of unscaling and reading found_inf on the
host. The kernel divides each gradient by the scale and, when found_inf is set, writes nothing; the
capturable step counts advanced before the launch are set back by found_inf after it (torch's fused
AdamW does the same). The non-capturable form reads found_inf once on the host (as GradScaler's own
skip does) so its host step counts stay exact.

Parameters must be fp32 CUDA tensors with dense, contiguous gradients; anything else raises
(there is no CPU fallback).
"""
from __future__ import annotations

import math
from typing import Iterable, Optional

import numpy as np
import torch

from . import _lib
from .ops import check

__all__ = ["AdamW"]

# rf_adamw_tensor (include/recformer_hip.h): 6 pointers, numel, first_block, 9 floats, 1 int
_DESC = np.dtype([("param", "<u8"), ("grad", "<u8"), ("exp_avg", "<u8"), ("exp_avg_sq", "<u8"), ("step", "<u8"),
                  ("hyper", "<u8"), ("numel", "<i8"), ("first_block", "<i8"), ("decay", "<f4"), ("beta1", "<f4"), ("w1", "<f4"),
                  ("beta2", "<f4"), ("w2", "<f4"), ("eps", "<f4"), ("lr", "<f4"), ("step_size", "<f4"),
                  ("bc2_sqrt", "<f4"), ("maximize", "<i4")])
assert _DESC.itemsize == 104


class _Plan:
    """One parameter subset's launch plan: the block -> tensor table and the last descriptors."""

    def __init__(self):
        self.table_key = None
        self.first: Optional[np.ndarray] = None
        self.table: Optional[np.ndarray] = None
        self.blob_key = None
        self.blob = None  # (pinned host copy, device copy) of the last descriptors
        self.spare = None  # pinned buffer reserved for a captured step's descriptors


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW's interface (lr, betas, eps, weight_decay, amsgrad=False, maximize),
    one rf_adamw_step launch per step()."""

    _step_supports_amp_scaling = True  # GradScaler hands grad_scale / found_inf (module docstring)

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, *, maximize: bool = False,
                 capturable: bool = False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad:
            raise NotImplementedError("recformer_amd.optim.AdamW: amsgrad is not supported")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=maximize, capturable=capturable))
        self._chunk: Optional[int] = None
        # launch plans (descriptor table + its host / device copies), one per parameter subset stepped:
        # None = every parameter (step()), or the id tuple of a step_params() subset
        self._plans = {}
        self._graph_blobs = []  # descriptor blobs a captured graph reads: kept for the optimizer's lifetime
        self._hyper = None  # device (groups, 2) fp32: lr, 1 - lr * weight_decay of each capturable group
        self._hyper_vals = None  # the host values last uploaded into _hyper
        self._launches = 0

    def _state(self, p: torch.Tensor, capturable: bool) -> dict:
        st = self.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device) if capturable else torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def _hyper_values(self):
        out = []
        for group in self.param_groups:
            lr = group["lr"]
            lr = float(lr) if isinstance(lr, torch.Tensor) else lr
            out.append((float(np.float32(lr)), float(np.float32(1 - lr * group["weight_decay"]))))
        return out

    def sync_hyper(self, device=None) -> bool:
        """Upload each group's (lr, 1 - lr * weight_decay) into the device tensor the capturable
        kernel reads, if they changed since the last upload (stream-ordered, from pinned memory; no
        host wait). Must not run while a stream captures; returns whether it copied."""
        vals = self._hyper_values()
        if self._hyper is not None and vals == self._hyper_vals:
            return False
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("recformer_amd.optim.AdamW: the learning rate changed since the last uncaptured "
                               "step; call sync_hyper() before capturing")
        if device is None:
            device = next(p.device for g in self.param_groups for p in g["params"])
        if self._hyper is None or self._hyper.shape[0] != len(vals) or self._hyper.device != device:
            self._hyper = torch.empty(len(vals), 2, dtype=torch.float32, device=device)
        host = torch.tensor(vals, dtype=torch.float32).pin_memory()
        self._hyper.copy_(host, non_blocking=True)
        self._hyper_vals = vals
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._run(None)
        return loss

    @torch.no_grad()
    def step_params(self, params) -> None:
        """The update of `params` alone (a subset of the groups' parameters, each updated as step() would):
        CapturedTrainStep steps a layer's parameters while the backward of the layers below still runs.
        No GradScaler interplay (grad_scale / found_inf are not read): the caller steps subsets only
        without a scaler."""
        if getattr(self, "grad_scale", None) is not None or getattr(self, "found_inf", None) is not None:
            raise RuntimeError("recformer_amd.optim.AdamW.step_params: not with a GradScaler")
        self._run(tuple(id(p) for p in params))

    def prepare_params(self, params) -> None:
        """Reserve step_params(params)'s launch plan outside a capture (the pinned buffer its captured
        descriptor copy replays from), so a graph may capture that subset's first step."""
        params = list(params)
        pl = self._plans.get(tuple(id(p) for p in params))
        if pl is None:
            pl = self._plans[tuple(id(p) for p in params)] = _Plan()
        if self._chunk is None:
            self._chunk = int(_lib.load().rf_adamw_chunk())
        size = len(params) * _DESC.itemsize + 4 * sum((p.numel() + self._chunk - 1) // self._chunk for p in params)
        if pl.spare is None or pl.spare.numel() < size:
            pl.spare = torch.empty(max(size, 1), dtype=torch.uint8, pin_memory=True)

    def _run(self, subset) -> None:
        lib = _lib.load()
        pl = self._plans.get(subset)
        if pl is None:
            pl = self._plans[subset] = _Plan()
        only = None if subset is None else set(subset)
        if self._chunk is None:
            self._chunk = int(lib.rf_adamw_chunk())
        chunk = self._chunk
        # GradScaler (torch.amp) with _step_supports_amp_scaling: device scale and inf flag
        grad_scale = getattr(self, "grad_scale", None)
        found_inf = getattr(self, "found_inf", None)
        if not any(g.get("capturable", False) for g in self.param_groups) and found_inf is not None:
            if float(found_inf) != 0.0:  # GradScaler's skip; host step counts must not advance
                return
            found_inf = None
        rows, device, dev_steps = [], None, []
        hyper_needed = any(g.get("capturable", False) for g in self.param_groups)
        if hyper_needed:
            self.sync_hyper()
        for gi, group in enumerate(self.param_groups):
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            cap = group.get("capturable", False)
            if isinstance(lr, torch.Tensor):
                lr = float(lr)
            for p in group["params"]:
                if p.grad is None or (only is not None and id(p) not in only):
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("AdamW does not support sparse gradients")
                if not p.is_cuda or p.dtype != torch.float32 or g.dtype != torch.float32:
                    raise ValueError("recformer_amd.optim.AdamW: parameters and gradients must be fp32 CUDA "
                                     f"tensors (got {p.dtype} on {p.device}, grad {g.dtype})")
                if not (p.is_contiguous() and g.is_contiguous()):
                    raise ValueError("recformer_amd.optim.AdamW: parameters and gradients must be contiguous")
                if device is None:
                    device = p.device
                elif p.device != device:
                    raise ValueError("recformer_amd.optim.AdamW: all parameters must be on one device")
                st = self._state(p, cap)
                if cap:
                    if not st["step"].is_cuda:
                        st["step"] = st["step"].to(p.device)
                    dev_steps.append(st["step"])
                    # lr / decay from the device hyper slot: not part of the descriptor key, so a
                    # scheduler's new value needs no descriptor upload
                    step_ptr, hyper_ptr, step_size, bc2s, lr_d, dec_d = (st["step"].data_ptr(),
                                                                         self._hyper[gi].data_ptr(), 0.0, 1.0, 0.0, 1.0)
                else:
                    st["step"] += 1
                    step = float(st["step"])
                    step_ptr, hyper_ptr, step_size, bc2s = 0, 0, lr / (1 - b1 ** step), math.sqrt(1 - b2 ** step)
                    lr_d, dec_d = lr, 1 - lr * wd
                rows.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             step_ptr, hyper_ptr, p.numel(), dec_d, b1, 1 - b1, b2, 1 - b2, eps, lr_d, step_size,
                             bc2s, 1 if group["maximize"] else 0))
        if not rows:
            return
        if dev_steps:
            torch._foreach_add_(dev_steps, 1.0)
        numels = tuple(r[6] for r in rows)
        if numels != pl.table_key:
            nblk = np.array([(n + chunk - 1) // chunk for n in numels], dtype=np.int64)
            pl.first = np.concatenate([[0], np.cumsum(nblk)[:-1]]).astype(np.int64)
            pl.table = np.repeat(np.arange(len(numels), dtype=np.int32), nblk)
            pl.table_key = numels
        stream = torch.cuda.current_stream(device).cuda_stream
        capturing = torch.cuda.is_current_stream_capturing()
        key = tuple(rows) if dev_steps else None
        if key is not None and key == pl.blob_key:
            # capturable and nothing changed: the device descriptors of the last step stand (no copy,
            # so nothing host-side enters a captured graph)
            base, nd = pl.blob[1].data_ptr(), len(rows)
        else:
            d = np.zeros(len(rows), dtype=_DESC)
            cols = list(zip(*rows))
            names = ("param", "grad", "exp_avg", "exp_avg_sq", "step", "hyper", "numel", "decay", "beta1", "w1",
                     "beta2", "w2", "eps", "lr", "step_size", "bc2_sqrt", "maximize")
            for name, col in zip(names, cols):
                d[name] = col
            d["first_block"] = pl.first
            # one host->device copy: descriptors then the block -> tensor table, from pinned memory kept
            # with the device copy (a captured graph replays the copy from it). Pinned memory cannot be
            # allocated while a stream captures: uncaptured steps stage through a fresh pinned tensor
            # (torch's host allocator guards its reuse) and keep one spare, unused buffer for a capture.
            blob = np.concatenate([d.view(np.uint8), pl.table.view(np.uint8)])
            if capturing:
                host = pl.spare
                if host is None or host.numel() < blob.size:
                    raise RuntimeError("recformer_amd.optim.AdamW: run one uncaptured step before capturing")
                pl.spare = None
                host = host[: blob.size]
                host.numpy()[:] = blob
            else:
                host = torch.from_numpy(blob).pin_memory()
                if pl.spare is None or pl.spare.numel() < blob.size:
                    pl.spare = torch.empty(blob.size, dtype=torch.uint8, pin_memory=True)
            dev_blob = torch.empty(blob.size, dtype=torch.uint8, device=device)
            dev_blob.copy_(host, non_blocking=True)
            pl.blob, pl.blob_key = (host, dev_blob), key
            base, nd = dev_blob.data_ptr(), len(rows)
        if capturing and not any(b is pl.blob for b in self._graph_blobs):
            # a graph replays from these (the pinned source of its descriptor copy, or the device
            # descriptors it reuses): neither may return to torch's caching allocators while the
            # optimizer lives, whatever later uncaptured steps do with the plan's blob
            self._graph_blobs.append(pl.blob)
        gs = grad_scale.data_ptr() if grad_scale is not None else 0
        fi = found_inf.data_ptr() if found_inf is not None else 0
        for t in (grad_scale, found_inf):
            if t is not None and (t.dtype != torch.float32 or t.device != device or t.numel() != 1):
                raise ValueError("recformer_amd.optim.AdamW: grad_scale / found_inf must be fp32 scalars on the "
                                 "parameters' device")
        check(lib.rf_adamw_step_amp(base, nd, base + nd * _DESC.itemsize, int(pl.table.size), gs, fi, stream),
              "rf_adamw_step")
        if dev_steps and found_inf is not None:
            torch._foreach_sub_(dev_steps, [found_inf] * len(dev_steps))  # a skipped step is not counted
        self._launches += 1
