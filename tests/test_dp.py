"""Data-parallel path on CPU: world_size-2 gloo process groups.

Each rank takes its shard of a ragged C1 batch (recformer_amd.dp.shard_batch), encodes and
scores it with the CPU oracle standing in for the device encoder (the kernels themselves are
covered by the -m gpu tests), gathers the score rows, and the result must equal the
single-process full-batch scores bit for bit; the max-over-ranks timing helper is checked too.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from recformer_amd import dp


class _Arr:
    """A tensor sent through a multiprocessing queue by value (numpy), not as a shared-memory
    handle: torch's handle is only valid while the sending worker lives, and a worker that has
    already exited makes the parent's unpickle fail with ConnectionResetError."""

    def __init__(self, t):
        self.a = t.detach().cpu().numpy()


def _plain(x):
    if torch.is_tensor(x):
        return _Arr(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v) for v in x)
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    return x


def _unplain(x):
    if isinstance(x, _Arr):
        return torch.from_numpy(x.a)
    if isinstance(x, (list, tuple)):
        return type(x)(_unplain(v) for v in x)
    if isinstance(x, dict):
        return {k: _unplain(v) for k, v in x.items()}
    return x


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for n in (0, 1, 5, 8, 64, 67):
        for ws in (1, 2, 3, 8):
            spans = [dp.shard_range(n, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(ws - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        dp.shard_range(4, 2, 2)


def test_shard_batch_views():
    b = {"input_ids": torch.arange(10).view(5, 2), "labels": torch.arange(5)}
    s = dp.shard_batch(b, 1, 2)
    assert s["input_ids"].tolist() == [[6, 7], [8, 9]] and s["labels"].tolist() == [3, 4]
    with pytest.raises(ValueError):
        dp.shard_batch({"a": torch.zeros(3), "b": torch.zeros(4)}, 0, 2)


def _scores_for(batch):
    from oracle import restatement as R
    from tests.common import C1, hashed_model
    m = hashed_model(C1, seed=1)
    cfg = m.config
    _, z = R.model_forward(m.state_dict(), cfg, **batch)
    items = torch.linspace(-1, 1, 37 * cfg.hidden_size).view(37, cfg.hidden_size).sin()
    return R.cosine_scores(z, items, cfg.temp)


def _worker(rank, ws, port, B, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from recformer_amd.synth import synth_batch
        torch.set_num_threads(1)
        full = synth_batch(B, 256, 1000, seed=7, lens=[256, 200, 131, 77, 256][:B])
        mine = dp.shard_batch(full, rank, ws)
        local = _scores_for(mine)
        gathered = dp.gather_rows(local, B)
        t = dp.max_over_ranks(float(rank + 1))
        if rank == 0:
            out_q.put(_plain((gathered, t)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [4, 5])
def test_dp_gloo_world2_matches_single_process(B):
    from recformer_amd.synth import synth_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, tmax = _unplain(q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = synth_batch(B, 256, 1000, seed=7, lens=[256, 200, 131, 77, 256][:B])
    torch.set_num_threads(1)
    ref = _scores_for(full)
    assert gathered.shape == ref.shape
    # rows are computed independently; only BLAS blocking over the batch differs
    assert torch.allclose(gathered, ref, atol=1e-5, rtol=0)
    assert tmax == 2.0


def _grad_worker(rank, ws, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 4))
        x = torch.randn(8, 16)[rank * 4:(rank + 1) * 4]  # this rank's shard of one global batch
        loss = net(x).pow(2).mean()
        loss.backward()
        n = dp.allreduce_grads(list(net.parameters()), bucket_bytes=1024)
        if rank == 0:
            out_q.put(_plain(([p.grad.clone() for p in net.parameters()], n)))
    finally:
        dist.destroy_process_group()


def test_allreduce_grads_matches_full_batch():
    """world-2 data parallel: the averaged per-shard gradients equal the full-batch gradient."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    grads, n = _unplain(q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 4))
    x = torch.randn(8, 16)
    net(x).pow(2).mean().backward()
    for g, p in zip(grads, net.parameters()):
        assert torch.allclose(g, p.grad, atol=1e-6)
    assert n >= 2  # 1 KiB buckets force more than one collective


def _pretrain_worker(rank, ws, port, out_q, bucketed):
    """One rank of data-parallel pretraining's contrastive head (models.py:472-497): z from a
    shared projection of this rank's half batch, the all-gather keeping the local slot's graph,
    gradients averaged by dp.GradBucketer (during backward) or dp.allreduce_grads (after)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        out = _pretrain_step(rank, ws, bucketed)
        if rank == 0:
            out_q.put(_plain(out))
        else:
            out_q.put(_plain(None))
    finally:
        dist.destroy_process_group()


def _pretrain_step(rank, ws, bucketed):
    import types

    from recformer_amd import models
    from recformer_amd.config import RecformerConfig
    torch.manual_seed(0)
    proj = torch.nn.Sequential(torch.nn.Linear(24, 32), torch.nn.Tanh(), torch.nn.Linear(32, 16))
    xa, xb = torch.randn(6, 24), torch.randn(6, 24)
    B = 6 // ws
    xa, xb = xa[rank * B:(rank + 1) * B], xb[rank * B:(rank + 1) * B]
    bucketer = dp.GradBucketer(proj.parameters(), bucket_bytes=1024) if bucketed else None
    z1, z2 = proj(xa), proj(xb)
    z1.retain_grad()
    z2.retain_grad()
    stub = types.SimpleNamespace(config=RecformerConfig(hidden_size=16, temp=0.05), training=True, lm_head=None)
    outs = types.SimpleNamespace(hidden_states=None, attentions=None, global_attentions=None)
    res = models._pretrain_train_losses(stub, z1, z2, outs, None, None, None, None, B)
    res.loss.backward()
    n = bucketer.finish() if bucketed else dp.allreduce_grads(list(proj.parameters()), bucket_bytes=1024)
    return (float(res.loss), int(res.cl_correct_num), z1.grad.clone(), z2.grad.clone(),
            [p.grad.clone() for p in proj.parameters()], n)


@pytest.mark.parametrize("bucketed", [False, True])
def test_pretrain_contrastive_dp_world2_matches_single_process(bucketed):
    """world-2 gloo pretraining step (models.py:474-490 all_gather of z; local slot keeps its graph):
    every rank's loss and correct count equal one process on the whole batch; each rank's dL/dz is
    that process's gradient for its rows; the averaged parameter gradients are the single-process
    ones / world size (the reference's DDP averaging of identical global losses)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pretrain_worker, args=(r, 2, port, q, bucketed)) for r in range(2)]
    for p in procs:
        p.start()
    got = [_unplain(q.get(timeout=300)) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    loss, correct, gz1, gz2, grads, n = [g for g in got if g is not None][0]
    ref_loss, ref_correct, rz1, rz2, ref_grads, _ = _pretrain_step(0, 1, False)
    assert loss == pytest.approx(ref_loss, rel=1e-6)
    assert correct == ref_correct
    assert torch.allclose(gz1, rz1[:3], atol=1e-6) and torch.allclose(gz2, rz2[:3], atol=1e-6)
    for g, r in zip(grads, ref_grads):
        assert torch.allclose(g * 2, r, atol=1e-5, rtol=1e-5)
    assert n >= 2


def _accum_net():
    torch.manual_seed(0)
    # a side branch used only by some micro-batches: its parameters get no gradient on a rank whose
    # window never takes it (the data-dependent case of the global-attention projections)
    return torch.nn.ModuleDict({"a": torch.nn.Linear(16, 32), "b": torch.nn.Linear(32, 4),
                                "side": torch.nn.Linear(16, 32)})


def _accum_loss(net, x, use_side):
    h = torch.nn.functional.gelu(net["a"](x))
    if use_side:
        h = h + net["side"](x)
    return net["b"](h).pow(2).mean()


def _accum_data():
    g = torch.Generator().manual_seed(5)
    return torch.randn(3, 8, 16, generator=g)  # 3 micro-batches x 8 rows (4 per rank)


def _accum_worker(rank, ws, port, out_q):
    """Gradient accumulation over 3 micro-batches with GradBucketer.no_sync (finetune.py:112-126):
    the side branch is taken only by rank 0's last micro-batch."""
    import contextlib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        net = _accum_net()
        xs = _accum_data()
        b = dp.GradBucketer(net.parameters(), bucket_bytes=2048)
        nb = len(b.buckets)
        for i in range(3):
            x = xs[i, rank * 4:(rank + 1) * 4]
            with b.no_sync() if i < 2 else contextlib.nullcontext():
                (_accum_loss(net, x, use_side=(rank == 0 and i == 2)) / 3).backward()
        n = b.finish()
        during = b.collectives  # every collective of the window, the no_sync passes included
        grads = [p.grad.clone() for p in net.parameters()]
        # a second window that forgets no_sync must raise, not drop a micro-batch
        raised = False
        try:
            for i in range(2):
                _accum_loss(net, xs[i, rank * 4:(rank + 1) * 4], False).backward()
        except RuntimeError:
            raised = True
        out_q.put(_plain((rank, grads if rank == 0 else None, n, nb, during, raised)))
    finally:
        dist.destroy_process_group()


def test_gradbucketer_accumulation_world2():
    """world-2 gloo, 3 micro-batches, one finish(): the averaged gradients equal one process
    accumulating the whole 3 x 8 batch; exactly one collective per bucket per window (none during
    the no_sync passes); a rank-dependent unused parameter does not reorder the collectives."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_accum_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (_unplain(q.get(timeout=300)) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    grads, n, nb, during, raised = got[0]
    assert nb >= 3 and n == nb and got[1][1] == nb
    assert during == nb and got[1][3] == nb
    assert raised and got[1][4]
    net = _accum_net()
    xs = _accum_data()
    for i in range(3):
        # rank 0's rows take the side branch in the last micro-batch, rank 1's do not
        l0 = _accum_loss(net, xs[i, :4], use_side=(i == 2))
        l1 = _accum_loss(net, xs[i, 4:], use_side=False)
        ((l0 + l1) / 2 / 3).backward()
    for g, p in zip(grads, net.parameters()):
        assert torch.allclose(g, p.grad, atol=1e-6, rtol=1e-5)


def _wire_net():
    torch.manual_seed(3)
    return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64),
                               torch.nn.GELU(), torch.nn.Linear(64, 8))


def _wire_worker(rank, ws, port, out_q):
    """Two windows per wire dtype: GradBucketer with .grad as bucket views, fp32 / bf16 / fp16 on the
    wire; the second window after optimizer-style zero_grad(set_to_none=True) (the hook re-binds)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        g = torch.Generator().manual_seed(9)
        xs = torch.randn(2, 8 * ws, 64, generator=g)
        res = {}
        for name, cd in (("fp32", None), ("bf16", torch.bfloat16), ("fp16", torch.float16)):
            net = _wire_net()
            # a warm-up backward before the bucketer exists: its gradients are kept (copied into the views)
            net(xs[1, :3]).sum().backward()
            pre = [p.grad.clone() for p in net.parameters()]
            b = dp.GradBucketer(net.parameters(), bucket_bytes=16 << 10, comm_dtype=cd)
            flats = [(f.data_ptr(), f.data_ptr() + f.numel() * f.element_size()) for f in b._flat]
            kept = all(torch.equal(p.grad, g0) and any(a <= p.grad.data_ptr() < e for a, e in flats)
                       for p, g0 in zip(net.parameters(), pre))
            b.zero_grad()
            grads = []
            for w in range(2):
                if w == 1:
                    for p in net.parameters():
                        p.grad = None  # optimizer.zero_grad(set_to_none=True)
                x = xs[w, rank * 8:(rank + 1) * 8]
                net(x).pow(2).mean().backward()
                b.finish()
                aliased = all(any(a <= p.grad.data_ptr() < e for a, e in flats) for p in net.parameters())
                grads.append(([p.grad.clone() for p in net.parameters()], aliased))
                b.zero_grad()
            res[name] = (grads, b.bucket_bytes_on_wire(), len(b.buckets), kept)
        out_q.put(_plain((rank, res)))
    finally:
        dist.destroy_process_group()


def _run_wire(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wire_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    got = dict(_unplain(q.get(timeout=300)) for _ in range(ws))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def test_gradbucketer_16bit_wire_world2():
    """world-2 gloo: the 16-bit exchange (DeepSpeed precision=16's reduce, lightning_pretrain.py:134-145)
    averages the gradients to the 16-bit contract of the fp32 exchange, which equals the full-batch
    gradient; .grad stays a view into the bucket buffers (no flatten / copy-back), also after a
    set-to-None zero_grad; the wire carries half the bytes."""
    got = _run_wire(2)
    xs = torch.randn(2, 16, 64, generator=torch.Generator().manual_seed(9))
    for w in range(2):
        net = _wire_net()
        net(xs[w]).pow(2).mean().backward()
        full = [p.grad for p in net.parameters()]
        for r in (0, 1):
            res = got[r]
            g32, al32 = res["fp32"][0][w]
            assert al32
            for a, ref in zip(g32, full):
                assert torch.allclose(a, ref, atol=1e-6, rtol=1e-5)
            for name, eps in (("bf16", 2 ** -8), ("fp16", 2 ** -11)):
                g16, al = res[name][0][w]
                assert al
                for a, b32 in zip(g16, g32):
                    # pre-divide + 16-bit rounding of each rank's half + the 16-bit sum: <= 3 roundings
                    assert (a - b32).abs().max() <= 3 * eps * b32.abs().max() + 1e-12, name
    n32, n16 = got[0]["fp32"][1], got[0]["bf16"][1]
    assert n16 * 2 == n32 and got[0]["fp32"][2] >= 2
    # gradients present when the bucketer is built are kept in its views (advisor r05), every wire dtype
    assert all(got[r][name][3] for r in (0, 1) for name in ("fp32", "bf16", "fp16"))


@pytest.mark.parametrize("ws", [2, 4])
def test_gradbucketer_16bit_wire_error_vs_world_size(ws):
    """How the 16-bit exchange's error grows with the ranks: each rank's term t_r = g_r / ws
    is rounded once to 16 bits (pack), and the ring adds ws - 1 partial sums, each rounded to 16 bits.
    Per element, with S = sum_r |t_r| (the sum of the magnitudes entering the reduction):
        |g_16 - g_32| <= (ws + 1) * (eps / 2 * S + tiny),   eps = 2^-7 (bf16), 2^-10 (fp16)
    (pack: eps/2 * S; each of the ws - 1 additions: eps/2 * |partial| <= eps/2 * S; tiny = half the wire
    dtype's subnormal spacing per rounding, which matters for fp16 gradients below 6.1e-5). Checked at world 2 and
    4 on gloo, whose ring sums in the wire dtype like RCCL's; at world 8 the bound is 9 * eps / 2 * S
    (3.5% of S in bf16 worst case; the measured error is far below it: the roundings do not all align)."""
    got = _run_wire(ws)
    xs = torch.randn(2, 8 * ws, 64, generator=torch.Generator().manual_seed(9))
    worst = {"bf16": 0.0, "fp16": 0.0}
    for w in range(2):
        per_rank = []
        for r in range(ws):
            net = _wire_net()
            net(xs[w, r * 8:(r + 1) * 8]).pow(2).mean().backward()
            per_rank.append([p.grad / ws for p in net.parameters()])
        S = [sum(t[i].abs() for t in per_rank) for i in range(len(per_rank[0]))]
        for r in range(ws):
            g32 = got[r]["fp32"][0][w][0]
            for i, (a, ref) in enumerate(zip(g32, [sum(t[i] for t in per_rank) for i in range(len(S))])):
                assert torch.allclose(a, ref, atol=1e-6, rtol=1e-5)
            # tiny: half the spacing of the wire dtype's subnormals, per rounding (fp16's start below 6.1e-5)
            for name, eps, tiny in (("bf16", 2.0 ** -7, 2.0 ** -134), ("fp16", 2.0 ** -10, 2.0 ** -25)):
                g16 = got[r][name][0][w][0]
                for a, b32, s in zip(g16, g32, S):
                    err = (a - b32).abs()
                    lim = (ws + 1) * ((eps / 2) * s + tiny)
                    assert bool((err <= lim + 1e-30).all()), (name, ws, float((err / lim).max()))
                    worst[name] = max(worst[name], float((err / lim).max()))
    # the ranks agree bit for bit (every rank unpacks the same reduced wire)
    for name in ("fp32", "bf16", "fp16"):
        for r in range(1, ws):
            for a, b in zip(got[0][name][0][1][0], got[r][name][0][1][0]):
                assert torch.equal(a, b)
    print(f"world {ws}: max error / bound = {worst['bf16']:.3f} (bf16), {worst['fp16']:.3f} (fp16)")


def _combine_worker(rank, ws, port, out_q):
    """One rank's shard result for C5 retrieval (what rf_score_rank + rf_topk_* produce on the
    device): counts over its catalog shard and its top-k with global ids; combined over ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from recformer_amd.ranker import combine_shards
        parts = _shard_parts(rank, ws)
        out = combine_shards(parts, 5)
        out_q.put(_plain((rank, {k: (v.clone() if torch.is_tensor(v) else v) for k, v in out.items()})))
    finally:
        dist.destroy_process_group()


def _scores():
    g = torch.Generator().manual_seed(3)
    s = torch.round(torch.randn(6, 40, generator=g) * 4) / 4  # ties across shard boundaries
    lab = torch.tensor([0, 39, 17, 20, 5, 33])
    return s, lab


def _shard_parts(rank, ws):
    from recformer_amd.ranker import merge_topk
    s, lab = _scores()
    a, b = dp.shard_range(s.shape[1], rank, ws)
    sl = s.gather(1, lab[:, None])
    sh = s[:, a:b]
    ids = torch.arange(a, b, dtype=torch.int32).expand(s.shape[0], b - a)
    v, i = merge_topk(sh, ids, 5)
    return {"gt": (sh > sl).sum(1).to(torch.int32), "valid": torch.full((s.shape[0],), b - a, dtype=torch.int32),
            "sexp": torch.exp(sh - 20.0).sum(1), "topv": v, "topi": i, "shift": 20.0}


def test_retrieval_combine_world2_matches_one_shard():
    """world-2 gloo: each rank's catalog-shard counts and top-k (ties across the shard boundary),
    combined by ranker.combine_shards (all-reduce of counts / exp-sums, all-gather + merge of the
    top-k), equal the single-shard result on every rank."""
    from recformer_amd.ranker import merge_topk
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_combine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(_unplain(q.get(timeout=300)) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    s, lab = _scores()
    ref_v, ref_i = merge_topk(s, torch.arange(40, dtype=torch.int32).expand(6, 40), 5)
    for r in (0, 1):
        out = got[r]
        assert torch.equal(out["gt"], (s > s.gather(1, lab[:, None])).sum(1).to(torch.int32))
        assert torch.equal(out["valid"], torch.full((6,), 40, dtype=torch.int32))
        assert torch.allclose(out["sexp"], torch.exp(s - 20.0).sum(1), rtol=1e-6)
        assert torch.equal(out["topv"], ref_v) and torch.equal(out["topi"], ref_i)
