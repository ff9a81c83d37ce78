"""recformer_amd.graphs.CapturedTrainStep: a finetune training step (RecformerForSeqRec forward,
backward, AdamW; finetune.py:98-137) captured once as a HIP graph and replayed, against the same
steps run eagerly — identical losses and parameters without dropout; with attention-probability
dropout, replay k draws exactly the masks of an eager step whose device step counter is k (the
counter the graph advances), so fresh masks per replay and forward/backward agreement are pinned."""
import pytest
import torch

from recformer_amd import RecformerForSeqRec, _lib, graphs
from recformer_amd.optim import AdamW
from tests.common import C1, batch_of, hashed_model, load_golden

pytestmark = pytest.mark.gpu


def _model(dev, att_p=0.0):
    cfg = dict(C1, hidden_dropout_prob=0.0, attention_probs_dropout_prob=att_p)
    lf = hashed_model(cfg, seed=1)
    m = RecformerForSeqRec(lf.config)
    m.longformer.load_state_dict(lf.state_dict())
    m.config.finetune_negative_sample_size = 0
    torch.manual_seed(0)
    m.init_item_embedding(torch.randn(40, cfg["hidden_size"]) * 0.5)
    return m.to(dev).train()


def _batch(dev):
    g = load_golden("c1_full")
    b = {k: v.to(dev) for k, v in batch_of(g).items()}
    b["labels"] = torch.tensor([3, 17, 0, 39], device=dev)
    return b


def _eager_step(m, opt, batch, dtype):
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=dtype):
        loss = m(**batch)
    loss.backward()
    opt.step()
    return float(loss)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_captured_finetune_step_matches_eager(dev, dtype):
    batch = _batch(dev)
    a, b = _model(dev), _model(dev)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    step = graphs.CapturedTrainStep(a, oa, batch, autocast_dtype=dtype, warmup=2)
    losses = [_eager_step(b, ob, batch, dtype) for _ in range(2)]
    for _ in range(3):
        la = float(step())
        losses.append(_eager_step(b, ob, batch, dtype))
        assert abs(la - losses[-1]) <= 1e-5 * max(1.0, abs(la)), (la, losses[-1])
    assert losses[-1] < losses[0]  # it trains
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n
    assert float(next(iter(oa.state.values()))["step"]) == 5.0


def test_captured_step_dropout_masks_follow_device_counter(dev):
    batch = _batch(dev)
    a, b = _model(dev, att_p=0.1), _model(dev, att_p=0.1)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, capturable=True)
    # warmup (eager, host seeds) then capture (host seeds drawn next, mixed with the counter on every
    # replay): the eager model replays the same CPU-generator draws
    torch.manual_seed(123)
    step = graphs.CapturedTrainStep(a, oa, batch, warmup=1)
    torch.manual_seed(123)
    _eager_step(b, ob, batch, torch.bfloat16)
    st = torch.get_rng_state()
    lib = _lib.load()
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    got, ref = [], []
    for k in (1, 2):
        got.append(float(step()))
        counter.fill_(k)
        torch.set_rng_state(st)
        old = lib.rf_set_seed_source(counter.data_ptr())
        try:
            ref.append(_eager_step(b, ob, batch, torch.bfloat16))
        finally:
            lib.rf_set_seed_source(old)
    assert got == pytest.approx(ref, rel=1e-5), (got, ref)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6)
    # the masks change between replays: step 2 with counter 1 would differ
    m3 = _model(dev, att_p=0.1)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        torch.manual_seed(123)
        counter.fill_(1)
        old = lib.rf_set_seed_source(counter.data_ptr())
        try:
            l1 = float(m3(**batch))
            counter.fill_(2)
            torch.manual_seed(123)
            l2 = float(m3(**batch))
        finally:
            lib.rf_set_seed_source(old)
    assert l1 != l2


def test_captured_step_refuses_more_global_tokens(dev):
    batch = _batch(dev)
    m = _model(dev)
    opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-4, capturable=True)
    step = graphs.CapturedTrainStep(m, opt, batch, warmup=1)
    more = dict(batch)
    gm = batch["global_attention_mask"].clone()
    gm[0, : int(batch["attention_mask"][0].sum())] = 1
    more["global_attention_mask"] = gm
    with pytest.raises(ValueError):
        step(more)
    with pytest.raises(ValueError):
        graphs.CapturedTrainStep(m, torch.optim.SGD(m.parameters(), lr=0.1), batch)


def test_captured_pretrain_step_matches_eager(dev):
    """RecformerForPretraining (two views, MLM on both, contrastive; models.py:382-520) captured:
    the masked-LM head over the fixed-capacity row set (labelled rows first, ignored rows after)
    gives the eager step's loss and parameters."""
    from tests.common import hashed_pretrain, pretrain_inputs
    from tests.test_gpu_train import CFG
    g = load_golden("c1_pretrain")
    kw = {k: v.to(dev) for k, v in pretrain_inputs(g).items()}
    a, b = hashed_pretrain(CFG).to(dev).train(), hashed_pretrain(CFG).to(dev).train()
    oa = AdamW(a.parameters(), lr=1e-3, capturable=True)
    ob = AdamW(b.parameters(), lr=1e-3, capturable=True)
    step = graphs.CapturedTrainStep(a, oa, kw, warmup=1)
    assert step.mlm_cap is not None

    def eager():
        ob.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = b(**kw)
        out.loss.backward()
        ob.step()
        return float(out.loss)

    eager()
    for _ in range(2):
        la, lb = float(step()), eager()
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n


def _lin_sched(opt, warm=2, total=12):
    """The reference's linear warmup / decay schedule (optimization.py:7-19, litmodels.py:57-62):
    lr = 0 when it is built, so a graph that froze the capture-time lr would never train."""
    def lam(s):
        return s / max(1, warm) if s < warm else max(0.0, 1 - s / max(1, total))
    return torch.optim.lr_scheduler.LambdaLR(opt, lam)


def test_captured_step_follows_lr_scheduler(dev):
    """A host LR scheduler stepped between replays reaches the captured AdamW (device lr, synced
    before each replay): parameters equal an eager run with the same schedule, and the first steps
    (lr = 0) change nothing."""
    batch = _batch(dev)
    a, b = _model(dev), _model(dev)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    sa, sb = _lin_sched(oa), _lin_sched(ob)
    before = [p.detach().clone() for p in a.parameters()]
    step = graphs.CapturedTrainStep(a, oa, batch, warmup=1)  # warmup runs at lr = 0: a no-op step
    assert all(torch.equal(x, p) for x, p in zip(before, a.parameters()))
    _eager_step(b, ob, batch, torch.bfloat16)
    for _ in range(4):
        sa.step()
        sb.step()
        la, lb = float(step()), _eager_step(b, ob, batch, torch.bfloat16)
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    assert oa.param_groups[0]["lr"] == ob.param_groups[0]["lr"] > 0
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n
    assert not all(torch.equal(x, p) for x, p in zip(before, a.parameters()))


def test_captured_step_survives_uncaptured_optimizer_steps(dev):
    """The graph's AdamW descriptors stay valid after uncaptured optimizer steps that rebuild them
    (another parameter subset, fresh pinned staging buffers reused by later host allocations)."""
    batch = _batch(dev)
    a, b = _model(dev), _model(dev)
    pa_all = [p for p in a.parameters() if p.requires_grad]
    pb_all = [p for p in b.parameters() if p.requires_grad]
    oa = AdamW(pa_all, lr=1e-3, capturable=True)
    ob = AdamW(pb_all, lr=1e-3, capturable=True)
    step = graphs.CapturedTrainStep(a, oa, batch, warmup=1)
    _eager_step(b, ob, batch, torch.bfloat16)
    la = float(step())
    lb = _eager_step(b, ob, batch, torch.bfloat16)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb))
    # an uncaptured step over half of the gradients (new descriptors, new pinned staging), on both
    for opt, ps in ((oa, pa_all), (ob, pb_all)):
        opt.zero_grad(set_to_none=True)
        for i, p in enumerate(ps):
            if i % 2 == 0:
                p.grad = torch.full_like(p, 1e-3)
        opt.step()
    junk = [torch.full((1 << 16,), 0xAB, dtype=torch.uint8).pin_memory() for _ in range(8)]  # reuse the blocks
    for _ in range(2):
        la, lb = float(step()), _eager_step(b, ob, batch, torch.bfloat16)
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    del junk
    for (n, x), y in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6), n


def _eager_window(m, opt, scaler, batches, k, clip):
    """finetune.py:98-126 with Lightning's gradient_clip_val (lightning_pretrain.py:140): fp16
    autocast, loss / k, GradScaler, unscale + clip, scaler.step / update, zero_grad."""
    for i in range(k):
        with torch.autocast("cuda", dtype=torch.float16):
            loss = m(**batches[i])
        scaler.scale(loss / k).backward()
    scaler.unscale_(opt)
    torch.nn.utils.clip_grad_norm_([p for p in m.parameters() if p.grad is not None], clip, foreach=True)
    scaler.step(opt)
    scaler.update()
    opt.zero_grad(set_to_none=True)
    return float(loss)


def test_captured_fp16_gradscaler_accumulation_clip_matches_eager(dev):
    """The reference drivers' training mode captured (finetune.py:106-126, lightning_pretrain.py:
    137-142): fp16 autocast + GradScaler + 2 accumulated micro-batches + clip at 1.0. An initial
    scale of 2^40 overflows the fp16 backward, so the first windows find inf gradients: the captured
    step skips the update (parameters and AdamW step counts unchanged) and backs the scale off on
    the device exactly as the eager GradScaler loop; then it trains and matches the eager loop."""
    b0 = _batch(dev)
    b1 = dict(b0)
    b1["labels"] = torch.tensor([5, 1, 30, 2], device=dev)
    mbs = [b0, b1]
    a, b = _model(dev), _model(dev)
    oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
    kw = dict(init_scale=2.0 ** 40, backoff_factor=2.0 ** -12, growth_interval=3)
    sa, sb = torch.amp.GradScaler("cuda", **kw), torch.amp.GradScaler("cuda", **kw)
    # the capture's eager warmup window runs at the overflowing scale (a skipped step), as eager
    step = graphs.CapturedTrainStep(a, oa, b0, autocast_dtype=torch.float16, warmup=1, scaler=sa,
                                    accumulation_steps=2, max_grad_norm=1.0)
    # eager: the same warmup window (on b0 twice, as the capture's warmup replays the example batch)
    _eager_window(b, ob, sb, [b0, b0], 2, 1.0)
    assert float(sa.get_scale()) == float(sb.get_scale())
    skipped = 0
    for w in range(4):
        pa0 = [p.detach().clone() for p in a.parameters()]
        for i in range(2):
            la = float(step(mbs[i]))
        ran = step.optimizer_was_run()
        lb = _eager_window(b, ob, sb, mbs, 2, 1.0)
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (w, la, lb)
        assert float(sa.get_scale()) == float(sb.get_scale()), (w, sa.get_scale(), sb.get_scale())
        if not ran:
            skipped += 1
            assert all(torch.equal(x, p) for x, p in zip(pa0, a.parameters()))
        st_a = float(next(iter(oa.state.values()))["step"])
        st_b = float(next(iter(ob.state.values()))["step"])
        assert st_a == st_b, (w, st_a, st_b)
    assert skipped >= 1 and float(sa.get_scale()) <= 2.0 ** 17
    assert float(next(iter(oa.state.values()))["step"]) >= 1  # it stepped after backing off
    for (n, x), y in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6), n


@pytest.mark.parametrize("wire", [None, torch.bfloat16])
def test_captured_dp_step_nccl_single_rank(dev, wire):
    """The data-parallel step captured with its RCCL all-reduces (dp.GradBucketer launching bucketed
    collectives from the backward hooks of the window's last micro-batch; the first micro-batch under
    no_sync): a one-rank nccl group on the box, so the collectives really run inside the HIP graph;
    the averaged gradients (world 1: the gradients) give the eager steps' parameters. The semantic
    world-2 check is test_dp.py / test_gpu_pretrain.py (gloo). Runs in the suite's own process: the
    capture is thread-local (graphs.CAPTURE_MODE — the c10d watchdog polling the warmup collectives'
    events during a global-mode capture was what aborted this test once in round 4), the warmup is
    drained before capture, and the graphs are released by close() before the process group is
    destroyed."""
    import os
    import socket
    import torch.distributed as dist
    from recformer_amd.dp import GradBucketer
    assert not dist.is_initialized()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(dev))
    step = None
    try:
        batch = _batch(dev)
        if wire is not None:
            # eager: the bucketed 16-bit exchange hands back exactly the fp32 gradients rounded once
            e1, e2 = _model(dev), _model(dev)
            eb = GradBucketer([p for p in e1.parameters()], bucket_bytes=1 << 20, single_rank=True, comm_dtype=wire)
            for m in (e1, e2):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    m(**batch).backward()
            eb.finish()
            for (n, x), y in zip(e1.named_parameters(), e2.parameters()):
                if y.grad is not None:
                    assert torch.equal(x.grad, y.grad.to(wire).float()), (n, float((x.grad - y.grad).abs().max()))
            del e1, e2, eb
        a, b = _model(dev), _model(dev)
        oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, capturable=True)
        ob = AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, capturable=True)
        bk = GradBucketer([p for p in a.parameters()], bucket_bytes=1 << 20, single_rank=True, comm_dtype=wire)
        assert len(bk.buckets) > 1
        step = graphs.CapturedTrainStep(a, oa, batch, warmup=1, accumulation_steps=2, bucketer=bk)
        n0 = bk.collectives
        # the eager reference runs the same exchange (its own bucketer, same wire): the captured step must
        # replay exactly what the eager DP loop does
        bkb = GradBucketer([p for p in b.parameters()], bucket_bytes=1 << 20, single_rank=True, comm_dtype=wire)

        def eager():
            for i in range(2):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = b(**batch) / 2
                if i == 0:
                    with bkb.no_sync():
                        loss.backward()
                else:
                    loss.backward()
            bkb.finish()
            ob.step()
            bkb.zero_grad()

        eager()
        for _ in range(2):
            step(batch)
            step(batch)
            eager()
        # launched from Python at warmup and at capture only (n0 counts them); replays re-run the captured ones
        assert n0 >= 2 * len(bk.buckets)
        assert bk.collectives == n0
        tol = dict(rtol=1e-5, atol=1e-6)
        worst = sorted(((float((x - y).abs().max()), n) for (n, x), y in zip(a.named_parameters(), b.parameters())),
                       reverse=True)[:4]
        for (n, x), y in zip(a.named_parameters(), b.parameters()):
            assert torch.allclose(x, y, **tol), (n, worst)
        assert all(p.grad is None or any(f.data_ptr() <= p.grad.data_ptr() < f.data_ptr() + f.numel() * 4
                                         for f in bk._flat) for p in a.parameters())
        step.close()
        with pytest.raises(RuntimeError):
            step(batch)
    finally:
        if step is not None:
            step.close()  # the captured RCCL kernels go before their communicator
        dist.destroy_process_group()


@pytest.mark.parametrize("chunk", [1000, 1 << 30])
def test_overlapped_optimizer_bit_identical(dev, chunk, monkeypatch):
    """graphs.OVERLAP_OPTIMIZER: the AdamW update of each chunk of parameters whose gradients are final runs
    on a side stream during the backward (optim.AdamW.step_params); the parameters after the captured
    steps are bit-identical to the serial step's (small chunks: many launches beside the backward)."""
    batch = _batch(dev)
    res = []
    for on in (True, False):
        monkeypatch.setattr(graphs, "OVERLAP_OPTIMIZER", on)
        monkeypatch.setattr(graphs, "OPT_CHUNK", chunk)
        a = _model(dev)
        oa = AdamW([p for p in a.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01, capturable=True)
        step = graphs.CapturedTrainStep(a, oa, batch, warmup=2)
        assert (step._ov is not None) == on
        if on:
            assert len(step._ov["chunks"]) >= (2 if chunk == 1000 else 1)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        res.append([p.detach().clone() for p in a.parameters()])
        assert all(float(s["step"]) == 5.0 for s in oa.state.values())
        step.close()
    for pa, pb in zip(*res):
        assert torch.equal(pa, pb)
