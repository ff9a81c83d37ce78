"""HIP-graph replay: GraphedForward (inference forwards, small serving batches) and
CapturedTrainStep (a whole training step).

GraphedForward: an inference forward of `RecformerModel` / `RecformerForSeqRec` is ~150 kernel
launches, each preceded by Python argument checks and a ctypes call; at a few sequences per batch
the host side, not the GPU, sets the latency. It captures one forward for a fixed batch shape into a
HIP graph (torch.cuda.CUDAGraph, i.e. hipGraph on ROCm) and replays it: new inputs are copied into
the captured input buffers, one graph launch runs every kernel, and the outputs are the captured
output tensors (overwritten by each replay). The library never allocates, synchronises or reads back
inside a forward except for one host read of the number of global tokens per sequence
(models.RecformerModel._encode); during capture that count is fixed to the example batch's
(models._STATIC_GMAX). A replay batch with more global tokens per sequence than the example is
rejected (check=True reads the count back: one host read instead of ~150 launches).

CapturedTrainStep: a whole training step — forward, backward and the optimizer — captured once as a
HIP graph and replayed per batch (the reference runs every step eagerly through autograd: finetune.py:98-137,
lightning_pretrain.py). A C3/C4 step issues ~1500 launches through Python autograd; replaying the
captured graph removes that host work, so the step costs its GPU time.

What capture needs from the step, and how the build provides it:
  * no host reads of device values: the global-slot count (train.encode_train's gmax) is fixed at
    capture to the maximum over the example batch's global_attention_mask(s) (train._STATIC_GMAX);
    a later batch may have fewer global tokens (empty slots are inert) but not more — __call__
    checks that unless check=False;
  * the masked-LM head over a fixed number of rows (models._STATIC_MLM_ROWS): the labelled rows
    first, padded with ignored rows up to a capacity of 1.25x the example's count (mlm_slack), so
    batches with up to that many labelled tokens per view replay the same graph;
  * fresh dropout masks on every replay: a device step counter registered with rf_set_seed_source
    is advanced inside the graph; every dropout kernel mixes it into its (capture-time) seed, and the
    backward regenerates the forward's masks from the same counter value (torch's own dropout, e.g.
    after the embeddings, uses its graph-safe philox offsets);
  * an optimizer without host state: recformer_amd.optim.AdamW(capturable=True) (device step
    counts, bias corrections in the kernel);
  * static inputs: the batch is copied into the graph's input buffers before each replay.
Gradients are written (not accumulated) by each replay; the graph owns them (with a dp.GradBucketer the
bucket views are the gradients: accumulated into by the backward and zeroed after the optimizer).
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Dict, Optional

import torch

from . import _lib, dropout, models, train

__all__ = ["GraphedForward", "CapturedTrainStep", "static_gmax"]

# Stream-capture mode of every graph captured here. "thread_local" restricts the capture-unsafe HIP calls
# to the capturing thread only: in "global" mode (torch's default) a capture-unsafe call from ANY thread
# fails and invalidates the capture — and ProcessGroupNCCL's watchdog thread polls the events of the
# collectives launched before the capture (the captured step's eager warmup windows) with
# hipEventQuery until it reaps them. When that poll fell inside the capture, the query failed, the
# watchdog thread raised, and its exception terminated the process while the main thread sat in
# capture_end (the round-4 abort of the captured one-rank RCCL step, gpurun_out/r04f2/pytest.log).
CAPTURE_MODE = "thread_local"
# CapturedTrainStep's backward with the weight gradients deferred to the side stream (train.deferred_weight_grads):
# off — measured slower (captured C3 17.04 vs 15.77 ms in one process, gpurun_out/r06k: the dW GEMMs then
# queue up beside the main stream's kernels, which the per-Linear join used to pace, and the end-of-backward
# join waits for the whole queue)
DEFER_DW = False
# the optimizer update overlapped with the backward (CapturedTrainStep without a scaler, clipping,
# accumulation or a DP bucketer): a parameter whose gradient is final (its post-accumulate hook, fired
# once per backward) joins a pending set; every OPT_CHUNK elements the set is updated on a side stream
# (optim.AdamW.step_params) while the backward of the layers below still runs, the rest after the
# backward. Same kernel, same per-element arithmetic: the parameters are bit-identical to the serial step.
# Off: measured slower (captured C3 16.24 vs 15.74 ms in one process, profiles/r06/c3_ab_overlap_opt.txt):
# the HBM-bound update's workgroups take CUs from the backward's persistent GEMMs on the critical path
OVERLAP_OPTIMIZER = False
OPT_CHUNK = 4 << 20


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
        # the CLS-only last layer (models._cls_last_layer) of pooled-only callers is captured when the
        # example has a global CLS in every sequence; replays are then checked for the same
        self.cls_global = static_cls_global(self.static)
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        old, old_c = models._STATIC_GMAX, models._STATIC_CLS
        try:
            models._STATIC_GMAX = self.gmax
            models._STATIC_CLS = self.cls_global
            with torch.no_grad():
                with torch.cuda.stream(stream):  # warm-up: caches, packed weights, kernel attributes
                    for _ in range(max(1, warmup)):
                        module(**self.static)
                torch.cuda.current_stream().wait_stream(stream)
                self.graph = torch.cuda.CUDAGraph()
                torch.cuda.synchronize()
                with torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
                    self.out = module(**self.static)
        finally:
            models._STATIC_GMAX, models._STATIC_CLS = old, old_c
        lf = getattr(module, "longformer", module)
        self.cls_global = self.cls_global and bool(getattr(lf, "_last_pruned", False))

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
        if self.check and self.cls_global and not static_cls_global(self.static):
            raise ValueError("GraphedForward: captured with a global CLS token in every sequence (the CLS-only "
                             "last layer); this batch has a sequence without one")
        self.graph.replay()
        return self.out


def static_gmax(batch: Dict[str, torch.Tensor]) -> int:
    """Largest number of global tokens in any sequence of any view of the batch (host read)."""
    g = 0
    for k, v in batch.items():
        if k.startswith("global_attention_mask") and torch.is_tensor(v):
            am = batch.get("attention_mask" + k[len("global_attention_mask"):])
            gm = v != 0
            if am is not None:
                gm = gm & (am > 0)
            if gm.numel():
                g = max(g, int(gm.sum(1).max()))
    return g


def static_cls_global(batch: Dict[str, torch.Tensor]) -> bool:
    """Whether position 0 is a (valid) global token in every sequence of every view (host read): the
    condition for the CLS-only last layer (train._GlobalCLS)."""
    seen = False
    for k, v in batch.items():
        if k.startswith("global_attention_mask") and torch.is_tensor(v):
            am = batch.get("attention_mask" + k[len("global_attention_mask"):])
            gm = v[:, 0] != 0
            if am is not None:
                gm = gm & (am[:, 0] > 0)
            if not bool(gm.all()):
                return False
            seen = True
    return seen


def mlm_rows(batch: Dict[str, torch.Tensor]) -> int:
    """Largest number of labelled masked-LM tokens in any view of the batch (host read)."""
    n = 0
    for k, v in batch.items():
        if k.startswith("mlm_labels") and torch.is_tensor(v):
            n = max(n, int((v != -100).sum()))
    return n


def _default_loss(model, batch):
    return model(**batch)


def _split_output(out):
    """(loss, the model output object or None): loss_fn may return the loss or an output with .loss."""
    return (out, None) if torch.is_tensor(out) else (out.loss, out)


def _detached(obj):
    """A copy of a model output whose tensor fields are detached: keeping the output object itself
    would keep its autograd graph (and that graph's AccumulateGrad nodes, bound to the stream that
    created them) alive into the next capture."""
    if obj is None:
        return None
    if dataclasses.is_dataclass(obj):
        return dataclasses.replace(obj, **{f.name: getattr(obj, f.name).detach() for f in dataclasses.fields(obj)
                                           if torch.is_tensor(getattr(obj, f.name))})
    return None


class CapturedTrainStep:
    """step = CapturedTrainStep(model, optimizer, example_batch); loss = step(batch)

    optimizer: recformer_amd.optim.AdamW(..., capturable=True). loss_fn(model, batch) -> scalar
    loss or an output with .loss (default: model(**batch)); `output` keeps the captured last
    micro-batch's output object (e.g. RecformerForPretraining's cl_correct_num, a device tensor each
    replay overwrites). autocast_dtype: the autocast dtype of the step
    (None: fp32). warmup eager optimizer steps run on a side stream first (they are real training
    steps, with the same scaler / accumulation / clipping as the captured ones).

    The reference drivers' full training mode (finetune.py:98-137; lightning_pretrain.py:134-145:
    precision=16, accumulate_grad_batches, gradient_clip_val=1.0, data-parallel):
      scaler: a torch.amp.GradScaler — the loss is scaled before backward, the inf/NaN check, the
        AdamW's unscale and skip (optim.AdamW reads the scaler's device grad_scale / found_inf) and
        the scale update (torch._amp_update_scale_) are all device work inside the graph; a step
        with an inf gradient changes no parameter and backs the scale off on replay exactly as the
        eager GradScaler loop does.
      accumulation_steps k: each call runs ONE micro-batch (loss / k, as finetune.py:112-113); the
        k-th call of a window also runs the optimizer. Two graphs share one memory pool: the first
        k-1 micro-batches replay an accumulate-only graph (gradients added in place into .grad
        buffers that persist across replays), the k-th replays a graph with the micro-batch, the
        gradient exchange, clipping, the optimizer step and the in-place zeroing of the gradients.
      max_grad_norm: torch.nn.utils.clip_grad_norm_ after unscaling (Lightning's
        gradient_clip_val): device-side norm and scale, no host read.
      bucketer: a dp.GradBucketer — its bucketed all-reduces are launched from the backward hooks
        of the window's last micro-batch and captured with it (RCCL collectives inside the graph,
        overlapped with that backward); the other micro-batches run under its no_sync().
    After the window's last call, `found_inf` (device scalar, 1.0 when the step was skipped) and
    `optimizer_was_run()` (host read) tell a driver whether to step its LR scheduler, as
    finetune.py:119-125 does with the scaler's scale; the optimizer's learning rates are re-read
    from its param_groups (optim.AdamW.sync_hyper) before every replay, so a host LR scheduler
    works unchanged."""

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, example: Dict[str, torch.Tensor],
                 loss_fn: Optional[Callable] = None, autocast_dtype: Optional[torch.dtype] = torch.bfloat16,
                 warmup: int = 3, mlm_slack: float = 1.25, scaler=None, accumulation_steps: int = 1,
                 max_grad_norm: Optional[float] = None, bucketer=None):
        if not all(g.get("capturable", False) for g in optimizer.param_groups):
            raise ValueError("CapturedTrainStep needs an optimizer constructed with capturable=True")
        if accumulation_steps < 1:
            raise ValueError(f"accumulation_steps must be >= 1, got {accumulation_steps}")
        if scaler is not None and not scaler.is_enabled():
            scaler = None
        self.model, self.opt = model, optimizer
        self.loss_fn = loss_fn or _default_loss
        self.dtype = autocast_dtype
        self.scaler, self.k, self.max_grad_norm, self.bucketer = scaler, int(accumulation_steps), max_grad_norm, bucketer
        self.params = [p for g in optimizer.param_groups for p in g["params"]]
        dev = next(model.parameters()).device
        self.static = {k: (v.to(dev).clone() if torch.is_tensor(v) else v) for k, v in example.items()}
        self.gmax = static_gmax(self.static)
        self.cls_global = static_cls_global(self.static)
        n = mlm_rows(self.static)
        self.mlm_cap = ((int(n * mlm_slack) + 63) // 64) * 64 if n else None
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.found_inf = None
        self.output = None
        self._pos = 0  # micro-batches run in the current accumulation window
        lib = _lib.load()
        self._ov = None
        if (OVERLAP_OPTIMIZER and scaler is None and max_grad_norm is None and bucketer is None and self.k == 1
                and hasattr(optimizer, "step_params") and all(p.is_leaf for p in self.params)):
            self._ov = {"on": False, "count": {}, "order": [], "chunks": None, "of": {}, "left": [],
                        "stepped": set(), "stream": torch.cuda.Stream(dev), "hooks": []}
            for p in self.params:
                if p.requires_grad:
                    self._ov["hooks"].append(p.register_post_accumulate_grad_hook(self._grad_ready))

        def micro(last: bool):
            """One micro-batch: forward, (scaled) backward; the last of a window also steps."""
            if self.dtype is None:
                loss, obj = _split_output(self.loss_fn(self.model, self.static))
            else:
                with torch.autocast("cuda", dtype=self.dtype, cache_enabled=False):
                    loss, obj = _split_output(self.loss_fn(self.model, self.static))
            self.output = _detached(obj)  # the captured output (e.g. cl_correct_num): changes per replay
            out = loss / self.k if self.k > 1 else loss
            if self.scaler is not None:
                out = self.scaler.scale(out)
            # the Linear weight gradients accumulate on the side stream with one join at the end of the
            # backward (train.DEFER_DW; DP bucketers' hooked parameters keep autograd's accumulation)
            ov = self._ov
            if ov is not None:
                # the first backward only records the order and count of the gradient accumulations;
                # afterwards the parameters accumulated exactly once are updated chunk by chunk as their
                # gradients become final
                ov["count"].clear()
                ov["order"].clear()
                ov["on"] = ov["chunks"] is not None
                if ov["on"]:
                    ov["left"] = [len(c) for c in ov["chunks"]]
                    ov["stepped"] = set()
            with train.deferred_weight_grads(DEFER_DW):
                if self.bucketer is not None and not last:
                    with self.bucketer.no_sync():
                        out.backward()
                else:
                    out.backward()
            if ov is not None and ov["chunks"] is None and not torch.cuda.is_current_stream_capturing():
                self._plan_chunks()
            if last:
                self._optimizer_part()
            if ov is not None:
                ov["on"] = False  # a backward outside the step (not this step's) must not update anything
            return loss

        def window():
            for i in range(self.k):
                micro(i == self.k - 1)

        old_g, old_m, old_c = train._STATIC_GMAX, models._STATIC_MLM_ROWS, train._STATIC_CLS
        train._STATIC_GMAX, models._STATIC_MLM_ROWS, train._STATIC_CLS = self.gmax, self.mlm_cap, self.cls_global
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self._zero_grads(set_to_none=True)
                    window()
                if self.bucketer is not None and self.bucketer.active:
                    # the bucket views are the persistent gradients the graphs accumulate into (zeroed
                    # by the step's graph after the optimizer, one fill per bucket)
                    self.bucketer.zero_grad()
                elif self.k > 1:
                    # persistent gradient buffers the accumulate graph adds into (zeroed by the last graph)
                    for p in self.params:
                        if p.requires_grad:
                            if p.grad is None:
                                p.grad = torch.zeros_like(p)
                            else:
                                p.grad.zero_()
                if hasattr(self.opt, "sync_hyper"):
                    self.opt.sync_hyper()
            torch.cuda.current_stream(dev).wait_stream(side)
            if self.k == 1 and not self._bucket_views():
                self.opt.zero_grad(set_to_none=True)
            # drain: every warmup kernel and collective finished before the capture starts (finish()
            # waited for the bucketer's handles on the stream; this waits for the device)
            torch.cuda.synchronize(dev)
            old_src = lib.rf_set_seed_source(self.counter.data_ptr())
            old_py = dropout.set_seed_counter(self.counter)
            try:
                self.graph_acc = None
                pool = None
                if self.k > 1:
                    self.graph_acc = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self.graph_acc, capture_error_mode=CAPTURE_MODE):
                        self.counter.add_(1)
                        self.loss_acc = micro(False).detach()
                    pool = self.graph_acc.pool()
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, pool=pool, capture_error_mode=CAPTURE_MODE):
                    self.counter.add_(1)
                    self.loss = micro(True).detach()
            finally:
                lib.rf_set_seed_source(old_src)
                dropout.set_seed_counter(old_py)
        finally:
            train._STATIC_GMAX, models._STATIC_MLM_ROWS, train._STATIC_CLS = old_g, old_m, old_c
        # the replay check on CLS-global batches only matters when the capture used the CLS-only layer
        lf = getattr(self.model, "longformer", self.model)
        self.cls_global = self.cls_global and bool(getattr(lf, "_last_pruned", False))
        self.replays = 0

    def _plan_chunks(self) -> None:
        """After the counting backward: the parameters accumulated exactly once, in accumulation order,
        cut into chunks of >= OPT_CHUNK elements; each chunk's launch plan is prepared now (outside any
        capture)."""
        ov = self._ov
        chunks, cur, n = [], [], 0
        for p in ov["order"]:
            if ov["count"][id(p)] != 1:
                continue
            cur.append(p)
            n += p.numel()
            if n >= OPT_CHUNK:
                chunks.append(cur)
                cur, n = [], 0
        if cur:
            chunks.append(cur)
        ov["chunks"] = chunks
        ov["of"] = {id(p): i for i, c in enumerate(chunks) for p in c}
        for c in chunks:
            self.opt.prepare_params(c)
        self.opt.prepare_params([p for p in self.params if id(p) not in ov["of"]])

    def _grad_ready(self, p: torch.Tensor) -> None:
        """Post-accumulate hook: p's gradient of this backward is complete (OVERLAP_OPTIMIZER)."""
        ov = self._ov
        if ov["chunks"] is None:
            ov["count"][id(p)] = ov["count"].get(id(p), 0) + 1
            if ov["count"][id(p)] == 1:
                ov["order"].append(p)
            return
        if not ov["on"]:
            return
        i = ov["of"].get(id(p))
        if i is None:
            return
        ov["left"][i] -= 1
        if ov["left"][i] == 0:  # the chunk's gradients are all final: update it beside the backward
            c = ov["chunks"][i]
            ov["stream"].wait_stream(torch.cuda.current_stream(p.device))
            with torch.cuda.stream(ov["stream"]):
                self.opt.step_params(c)
            ov["stepped"].add(i)

    def _optimizer_part(self):
        """Gradient exchange, unscale + clip, optimizer step, scale update, gradient zeroing."""
        ov = self._ov
        if ov is not None and ov["on"]:
            # overlapped: the parameters outside the chunks (a gradient accumulated more than once, or none
            # in the counting pass) here, a chunk that did not complete too, then the main stream joins
            # the side stream
            self.opt.step_params([p for p in self.params if id(p) not in ov["of"]])
            for i, c in enumerate(ov["chunks"]):
                if i not in ov["stepped"]:
                    self.opt.step_params(c)
            torch.cuda.current_stream(self.counter.device).wait_stream(ov["stream"])
            return
        if self.bucketer is not None:
            self.bucketer.finish()
        sc = self.scaler
        if self.max_grad_norm is not None:
            if sc is not None:
                sc.unscale_(self.opt)
            torch.nn.utils.clip_grad_norm_([p for p in self.params if p.grad is not None], self.max_grad_norm,
                                           foreach=True)
        if sc is not None:
            sc.step(self.opt)
            st = sc._per_optimizer_states[id(self.opt)]["found_inf_per_device"]
            self.found_inf = sum(v.to(sc._scale.device) for v in st.values())
            sc.update()
        else:
            self.opt.step()
        if self._bucket_views():
            self.bucketer.zero_grad()
        elif self.k > 1:
            torch._foreach_zero_([p.grad for p in self.params if p.grad is not None])

    def _bucket_views(self) -> bool:
        return self.bucketer is not None and self.bucketer.active

    def _zero_grads(self, set_to_none: bool):
        if self._bucket_views():
            self.bucketer.zero_grad()
        else:
            self.opt.zero_grad(set_to_none=set_to_none)

    def close(self):
        """Release the captured graphs (and the tensors they own) now, after the device has finished
        any replay: a graph with captured RCCL kernels must be torn down while its process group
        still exists, so a driver calls close() before dist.destroy_process_group() instead of
        leaving the graphs to the garbage collector. The step cannot be replayed afterwards."""
        if getattr(self, "graph", None) is None:
            return
        torch.cuda.synchronize(self.counter.device)
        if self._ov is not None:
            for h in self._ov["hooks"]:
                h.remove()
            self._ov = None
        for g in (self.graph_acc, self.graph):
            if g is not None:
                g.reset()
        self.graph = self.graph_acc = None
        self.loss = self.loss_acc = self.output = self.found_inf = None
        if self.bucketer is not None:
            self.bucketer.discard()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def optimizer_was_run(self) -> bool:
        """Whether the last completed window's optimizer step was taken (host read; True without a
        scaler)."""
        return self.found_inf is None or float(self.found_inf) == 0.0

    def __call__(self, batch: Optional[Dict[str, torch.Tensor]] = None, check: bool = True) -> torch.Tensor:
        """Copy batch (same shapes as the example) into the graph's inputs and replay one
        micro-batch (with accumulation_steps = 1: one whole step); returns the micro-batch's loss (a
        tensor the next replay overwrites)."""
        if batch is not None:
            if check:
                g = static_gmax(batch)
                if g > self.gmax:
                    raise ValueError(f"batch has {g} global tokens in a sequence; the step was captured for {self.gmax}")
                if self.cls_global and not static_cls_global(batch):
                    raise ValueError("the step was captured with a global CLS token in every sequence (the "
                                     "CLS-only last layer); this batch has a sequence without one")
                n = mlm_rows(batch)
                if n and (self.mlm_cap is None or n > self.mlm_cap):
                    raise ValueError(f"batch has {n} masked-LM labels in a view; the step was captured for {self.mlm_cap}")
            for k, v in batch.items():
                if torch.is_tensor(v):
                    dst = self.static[k]
                    if dst.shape != v.shape:
                        raise ValueError(f"{k}: shape {tuple(v.shape)} != captured {tuple(dst.shape)}")
                    dst.copy_(v, non_blocking=True)
        if self.graph is None:
            raise RuntimeError("CapturedTrainStep: replay after close()")
        self._pos += 1
        if self._pos < self.k:
            self.graph_acc.replay()
            self.replays += 1
            return self.loss_acc
        self._pos = 0
        if hasattr(self.opt, "sync_hyper"):
            self.opt.sync_hyper()  # the host's current learning rates (an LR scheduler's) into the graph
        self.graph.replay()
        self.replays += 1
        return self.loss
