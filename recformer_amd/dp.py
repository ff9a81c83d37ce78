"""Data-parallel plumbing for the encode+score path.

User sequences are independent, so inference shards a batch of sequences across ranks with
no data-path collective; the item catalog is replicated. The only collectives are host-side
bookkeeping: the max-over-ranks step time (bench) and, for evaluation drivers that want the
whole batch's scores on every rank, an all-gather of per-rank score rows in batch order
(the reference evaluates on one device, finetune.py:66-96, so the gathered result must equal
the single-device one row for row).

Works with any torch.distributed backend: `nccl` (RCCL over xGMI) on MI355X, `gloo` on CPU
(tests/test_dp.py).
"""
from __future__ import annotations

import contextlib
from typing import Dict, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    """(rank, world_size); (0, 1) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of n items for `rank` (sizes differ by at most 1,
    lower ranks take the remainder)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world {world_size}")
    q, r = divmod(n, world_size)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_batch(batch: Dict[str, torch.Tensor], rank: int, world_size: int) -> Dict[str, torch.Tensor]:
    """This rank's rows of every (B, ...) tensor in a collator batch dict (views, no copy)."""
    sizes = {v.shape[0] for v in batch.values() if torch.is_tensor(v) and v.dim() > 0}
    if len(sizes) != 1:
        raise ValueError(f"batch tensors disagree on the batch dimension: {sizes}")
    a, b = shard_range(sizes.pop(), rank, world_size)
    return {k: (v[a:b] if torch.is_tensor(v) and v.dim() > 0 else v) for k, v in batch.items()}


def max_over_ranks(x: float, device=None) -> float:
    """Max of a host scalar over all ranks (the bench's step time)."""
    rank, ws = world()
    if ws == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(local: torch.Tensor, total: int) -> torch.Tensor:
    """All-gather per-rank row blocks (from shard_batch's split of `total` rows) into the full
    (total, ...) tensor in the original row order, on every rank. Ragged shards are padded to
    the largest shard for the collective and trimmed after."""
    rank, ws = world()
    if ws == 1:
        return local
    q = -(-total // ws)
    a, b = shard_range(total, rank, ws)
    if local.shape[0] != b - a:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its shard is {b - a}")
    pad = local.new_zeros((q,) + tuple(local.shape[1:]))
    pad[: b - a] = local
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad.contiguous())
    out = []
    for r in range(ws):
        ra, rb = shard_range(total, r, ws)
        out.append(parts[r][: rb - ra])
    return torch.cat(out, 0)


def allreduce_grads(params, bucket_bytes: int = 64 << 20, average: bool = True) -> int:
    """Bucketed all-reduce of the parameter gradients over the default group (RCCL over xGMI
    with the nccl backend; gloo on CPU) — the data-parallel exchange of a training step
    (SURVEY.md §8e). Gradients are flattened per dtype into buckets of <= bucket_bytes, reduced
    with one collective each, and copied back; returns the number of collectives issued.
    (torch DistributedDataParallel over these modules does the same, overlapped with backward.)"""
    rank, ws = world()
    if ws == 1:
        return 0
    grads = [p.grad for p in params if p.grad is not None]
    n = 0
    by_dtype = {}
    for g in grads:
        by_dtype.setdefault((g.dtype, g.device), []).append(g)
    for (_, _), gs in by_dtype.items():
        bucket, size = [], 0
        for g in gs + [None]:
            if g is not None and (not bucket or size + g.numel() * g.element_size() <= bucket_bytes):
                bucket.append(g)
                size += g.numel() * g.element_size()
                continue
            if bucket:
                flat = torch.cat([b.reshape(-1) for b in bucket])
                dist.all_reduce(flat)
                if average:
                    flat /= ws
                off = 0
                for b in bucket:
                    b.copy_(flat[off:off + b.numel()].view_as(b))
                    off += b.numel()
                n += 1
            bucket, size = ([g], g.numel() * g.element_size()) if g is not None else ([], 0)
    return n


class GradBucketer:
    """Bucketed gradient all-reduce overlapped with backward (RCCL all-reduce of the
    gradients in ~25-50 MB buckets launched in reverse layer order during backward).

    Parameters are grouped, in reverse registration order (the order backward produces their
    gradients), into buckets of <= bucket_bytes per (dtype, device). Each bucket owns one persistent
    flat buffer and every parameter's .grad is a view into it (DDP's gradient_as_bucket_view): backward
    accumulates straight into the bucket, so there is no flattening copy before the collective and no
    copy back after it. A post-accumulate-grad hook counts each bucket's ready gradients; once a bucket
    is complete AND every lower-numbered bucket has been launched, its all-reduce is launched
    asynchronously, so communication of late layers overlaps the backward of early ones. Launches are
    strictly in bucket order on every rank — a bucket whose parameters got no gradient on one rank (e.g.
    the global-attention projections of a batch without global tokens) holds the later buckets back
    until `finish()` instead of letting ranks pair different buckets in the collective. `finish()`
    launches what is left, waits and averages (the mean of the ranks' gradients, as
    DistributedDataParallel); a parameter without a gradient on a rank contributes zeros. With one rank
    it does nothing (unless single_rank).

    comm_dtype: the dtype on the wire. None = the gradients' own (fp32 master gradients: 4 bytes per
    parameter, 592 MB per exchange at 148M parameters, averaged by the collective itself on RCCL);
    torch.bfloat16 / torch.float16 = a 16-bit exchange, as the reference's DeepSpeed precision=16 step
    (lightning_pretrain.py:134-145): each complete bucket is packed once into a 16-bit buffer, pre-divided
    by the world size (fp32 arithmetic, one rounding), all-reduced (296 MB per exchange), and unpacked
    into the fp32 bucket — fp32 master accumulation, a 16-bit exchange.

    Gradient storage: the bucket views are installed at construction and re-installed by zero_grad()
    (which zeroes the flat buffers: one fill per bucket). A driver that sets gradients to None
    (optimizer.zero_grad()) still works: the hook then copies the gradient autograd produced into its
    view once and re-binds .grad; a parameter that got no gradient in the window is zeroed in its view
    when its bucket is launched.

    Gradient accumulation (the reference accumulates 8 micro-batches per optimizer step under DDP,
    finetune.py:112-126, lightning_pretrain.py:137): run the first k-1 backward passes inside
    `no_sync()` (the hooks then do nothing and .grad accumulates locally), the last one outside, then
    `finish()` — one collective per bucket per optimizer step, as DDP's no_sync:

        b = GradBucketer(model.parameters())
        for i, batch in enumerate(micro_batches):
            with b.no_sync() if i < len(micro_batches) - 1 else contextlib.nullcontext():
                model(**batch).backward()
        b.finish(); opt.step(); b.zero_grad()

    A second backward outside `no_sync()` before `finish()` (its buckets may already be reduced)
    raises instead of silently dropping that micro-batch.

    Inside a captured training step (graphs.CapturedTrainStep(bucketer=...)) the hooks' packs and
    all-reduce launches and finish()'s waits and unpacks are recorded into the HIP graph, so each
    replay runs the RCCL collectives with the backward; the graph zeroes the buckets after the
    optimizer. single_rank=True keeps the collectives at world size 1 (a one-rank nccl group: the
    captured exchange on one GPU, tests).
    """

    def __init__(self, params, bucket_bytes: int = 32 << 20, average: bool = True, group=None,
                 single_rank: bool = False, comm_dtype: torch.dtype = None):
        self.rank, self.ws = world()
        if group is not None:
            self.rank, self.ws = dist.get_rank(group), dist.get_world_size(group)
        self.active = self.ws > 1 or (single_rank and dist.is_available() and dist.is_initialized())
        self.average = average
        self.group = group
        self.comm_dtype = comm_dtype
        if comm_dtype is not None and comm_dtype not in (torch.bfloat16, torch.float16):
            raise ValueError(f"comm_dtype must be None, torch.bfloat16 or torch.float16, got {comm_dtype}")
        self.params = [p for p in params if p.requires_grad]
        self.buckets = []
        self._handles = []
        self._sync = True
        self.collectives = 0  # collectives issued over the bucketer's lifetime (tests, logging)
        self.wire_bytes = 0   # bytes handed to the collectives over the bucketer's lifetime
        if not self.active:
            return
        by = {}
        for p in reversed(self.params):
            by.setdefault((p.dtype, p.device), []).append(p)
        for ps in by.values():
            cur, size = [], 0
            for p in ps:
                nb = p.numel() * p.element_size()
                if cur and size + nb > bucket_bytes:
                    self.buckets.append(cur)
                    cur, size = [], 0
                cur.append(p)
                size += nb
            if cur:
                self.buckets.append(cur)
        # one flat buffer per bucket, the .grad views into it, and the 16-bit wire buffer
        self._flat, self._views, self._wire = [], [], []
        self._of = {}
        for bi, ps in enumerate(self.buckets):
            flat = torch.zeros(sum(p.numel() for p in ps), dtype=ps[0].dtype, device=ps[0].device)
            views, off = [], 0
            for p in ps:
                views.append(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
                self._of[id(p)] = (bi, len(views) - 1)
                p.register_post_accumulate_grad_hook(self._hook)
            self._flat.append(flat)
            self._views.append(views)
            self._wire.append(torch.empty(flat.numel(), dtype=comm_dtype, device=flat.device)
                              if comm_dtype is not None and comm_dtype != flat.dtype else None)
        # average inside the collective where the backend has it (RCCL's ncclAvg), else divide after
        self._avg_op = None
        if average and self.ws > 1:
            try:
                if dist.get_backend(group) == "nccl":
                    self._avg_op = dist.ReduceOp.AVG
            except (RuntimeError, ValueError):
                self._avg_op = None
        # bind every .grad to its bucket view, keeping a gradient that is already there (a bucketer
        # built mid-accumulation or after a warm-up backward): copied in, not thrown away
        for ps, views in zip(self.buckets, self._views):
            for p, v in zip(ps, views):
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v
        self._reset()

    def _reset(self):
        self._ready = [0] * len(self.buckets)
        self._next = 0  # lowest bucket not yet launched
        self._seen = set()  # parameters whose gradient arrived in this window's synced backward

    def zero_grad(self):
        """Zero every bucket (one fill each) and bind each parameter's .grad to its bucket view — the
        optimizer.zero_grad() of a bucketed step (in-place, so the views stay the gradients)."""
        if not self.active:
            for p in self.params:
                if p.grad is not None:
                    p.grad.zero_()
            return
        for flat in self._flat:
            flat.zero_()
        for ps, views in zip(self.buckets, self._views):
            for p, v in zip(ps, views):
                if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                    p.grad = v

    def bucket_bytes_on_wire(self) -> int:
        """Bytes one exchange hands to the collectives (all buckets)."""
        if not self.active:
            return 0
        return sum(f.numel() * (w.element_size() if w is not None else f.element_size())
                   for f, w in zip(self._flat, self._wire))

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside accumulate into .grad with no collective (DDP.no_sync)."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _bind(self, bi):
        """Make every .grad of bucket bi its view: a gradient autograd put elsewhere (after a
        zero_grad(set_to_none=True)) is copied in once; a missing one is zero in the view."""
        for p, v in zip(self.buckets[bi], self._views[bi]):
            g = p.grad
            if g is None:
                v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def _hook(self, p):
        bi, j = self._of[id(p)]
        if not self._sync:
            g, v = p.grad, self._views[bi][j]
            if g is not None and g.data_ptr() != v.data_ptr():
                v.copy_(g)  # keep accumulating in the bucket view across no_sync micro-batches
                p.grad = v
            return
        if id(p) in self._seen:
            raise RuntimeError("GradBucketer: a second backward reached an already reduced bucket before finish(); "
                               "run all but the last micro-batch of an accumulation window under no_sync()")
        self._seen.add(id(p))
        self._ready[bi] += 1
        while self._next < len(self.buckets) and self._ready[self._next] >= len(self.buckets[self._next]):
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        self._bind(bi)
        flat, wire = self._flat[bi], self._wire[bi]
        if wire is not None:
            # pack: fp32 -> 16 bit, pre-divided by the world size (the mean's division before the sum)
            if self.average and self.ws > 1:
                torch.mul(flat, 1.0 / self.ws, out=wire)
            else:
                wire.copy_(flat)
            buf, op = wire, dist.ReduceOp.SUM
        else:
            buf, op = flat, (self._avg_op or dist.ReduceOp.SUM)
        self._handles.append((bi, dist.all_reduce(buf, op=op, group=self.group, async_op=True)))
        self.collectives += 1
        self.wire_bytes += buf.numel() * buf.element_size()

    def discard(self):
        """Forget this window's launched buckets without waiting (the work handles): a captured step's
        close() drops what its capture left behind."""
        self._handles = []
        if self.active:
            self._reset()

    def finish(self) -> int:
        """Wait for the window's buckets (launching, in bucket order, any not launched during
        backward), average, unpack a 16-bit exchange into the fp32 buckets; returns the number of
        collectives issued this window."""
        if not self.active:
            return 0
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        n = len(self._handles)
        for bi, h in self._handles:
            h.wait()
            flat, wire = self._flat[bi], self._wire[bi]
            if wire is not None:
                flat.copy_(wire)
            elif self.average and self.ws > 1 and self._avg_op is None:
                flat.div_(self.ws)
        self._handles = []
        self._reset()
        return n
