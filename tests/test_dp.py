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
            out_q.put((gathered, t))
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
    gathered, tmax = q.get(timeout=300)
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
            out_q.put(([p.grad.clone() for p in net.parameters()], n))
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
    grads, n = q.get(timeout=300)
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
