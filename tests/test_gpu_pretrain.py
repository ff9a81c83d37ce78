"""C4 pretraining at full model size (BASELINE configs[3]) on the HIP training path.

1. test_c4_pretrain_grads_match_reference — RecformerForPretraining (12L/768d, view a L=1024, view b
   L=128, MLM on both views, dropout 0) forward + backward against the REAL reference's pretraining
   step (tests/golden/c4_pretrain.npz, oracle/gen_golden_pretrain.py: models.py:370-520 incl.
   LongformerLMHead TF:1265-1285): loss, cl_correct_num, dL/dz of both views and, per parameter of
   the encoder AND the LM head, 256 gradient entries, the L2 norm and max-abs. fp32: as the C2
   finetune check (loss 1e-3, slices 2e-3 x max|g|, norms 1e-3). 16-bit autocast: loss 1e-2
   relative, dL/dz cosine >= 0.99, per-parameter slice cosine >= min(0.99, c_ref - 0.02) and norm
   within max(5%, |r_ref - 1| + 2%), where c_ref / r_ref are the cosine / norm ratio of the
   REFERENCE's own bf16-autocast gradients to its fp32 ones (stored in the fixture; fp16 runs with
   the loss scaled by 2^16 as GradScaler does in the reference's drivers): its
   value_global.bias gradients, for one, are only 0.97-0.99 cosine-close to fp32 in its own
   mixed-precision run, so a flat 0.99 would demand more than the reference achieves.
2. test_c4_pretrain_dp_world2 — the data-parallel step of lightning_pretrain.py (one process per
   rank, each on its share of the batch, z all-gathered with the local slot keeping its graph,
   models.py:474-490; gradients averaged as DDP does) with two real ranks over gloo sharing this
   GPU, each running the real 12-layer model with dp.GradBucketer: every rank's contrastive loss and
   correct count equal one process on the whole batch, the mean of the rank losses equals the
   single-process loss (equal masked-token counts per sequence make the per-rank MLM means average
   to the global one), and the averaged gradients equal the single-process gradients of
   loss - CL/2 (each rank back-propagates the full contrastive loss through its own slot only, so
   the average carries half of it: DDP's semantics for this loss, not a build choice).
"""
import contextlib
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FIX = os.path.join(HERE, "golden", "c4_pretrain.npz")
ALIAS = {"lm_head.decoder.bias": "lm_head.bias"}  # tied in the build (transformers 4.28 semantics)


def build_model(dev):
    from recformer_amd import RecformerConfig, RecformerForPretraining
    from recformer_amd.hashinit import hash_init_
    from recformer_amd.synth import BASE
    m = RecformerForPretraining(RecformerConfig(**dict(BASE, hidden_dropout_prob=0.0,
                                                       attention_probs_dropout_prob=0.0)))
    hash_init_(m.longformer, seed=2)
    hash_init_(m.lm_head, seed=7)
    return m.to(dev).train()


def fixture_inputs(gz, rows=None):
    keys = [k for k in gz.files if k.endswith("_a") or k.endswith("_b")]
    out = {k: torch.from_numpy(gz[k]) for k in keys}
    if rows is not None:
        out = {k: v[rows] for k, v in out.items()}
    return out


def _zero_grad_param(n):
    """Gradients that are mathematically zero: the key biases shift a softmax row uniformly."""
    return n.endswith("attention.self.key.bias") or n.endswith("attention.self.key_global.bias")


def _ref_drift(gz, n):
    """(cosine, norm ratio) of the reference's own bf16-autocast gradient slice to its fp32 one."""
    a, b = gz[f"gb:{n}:val"].astype(np.float64), gz[f"g:{n}:val"].astype(np.float64)
    cos = float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-300))
    return cos, float(gz[f"gb:{n}:norm"]) / float(gz[f"g:{n}:norm"])


def _ctx(mode):
    if mode == "fp32":
        return contextlib.nullcontext()
    return torch.autocast("cuda", dtype=torch.bfloat16 if mode == "autocast" else torch.float16)


@pytest.mark.parametrize("mode", ["fp32", "autocast", "autocast16"])
def test_c4_pretrain_grads_match_reference(dev, mode):
    gz = np.load(FIX)
    m = build_model(dev)
    zs = []

    def hook(_m, _i, out):
        if len(zs) < 2:
            out.pooler_output.retain_grad()
            zs.append(out.pooler_output)

    hdl = m.longformer.register_forward_hook(hook)
    batch = {k: v.to(dev) for k, v in fixture_inputs(gz).items()}
    with _ctx(mode):
        out = m(**batch)
    # fp16 runs as the reference's drivers run it: the loss scaled by GradScaler's initial 2^16
    # (finetune.py:106-126), the gradients unscaled before the comparison
    scale = 65536.0 if mode == "autocast16" else 1.0
    (out.loss * scale).backward()
    hdl.remove()
    if scale != 1.0:
        for p in m.parameters():
            if p.grad is not None:
                p.grad.div_(scale)
        for z in zs:
            z.grad.div_(scale)
    ref_loss = float(gz["loss"])
    assert int(out.cl_correct_num) == int(gz["cl_correct_num"])
    dz = [z.grad.float().cpu() for z in zs]
    dz_ref = [torch.from_numpy(gz["dz1"]), torch.from_numpy(gz["dz2"])]
    if mode == "fp32":
        assert abs(float(out.loss) - ref_loss) <= 1e-3, (float(out.loss), ref_loss)
        for a, b in zip(dz, dz_ref):
            assert float((a - b).abs().max()) <= 2e-3 * float(b.abs().max())
    else:
        assert abs(float(out.loss) - ref_loss) <= 1e-2 * abs(ref_loss), (float(out.loss), ref_loss)
        for a, b in zip(dz, dz_ref):
            assert F.cosine_similarity(a.reshape(1, -1), b.reshape(1, -1)).item() >= 0.99
    params = dict(m.named_parameters())
    names = [str(n) for n in gz["names"]]
    gmax = max(float(gz[f"g:{n}:maxabs"]) for n in names)
    checked = zero = 0
    for n in names:
        p = params[ALIAS.get(n, n)]
        assert p.grad is not None, n
        gr = p.grad.detach().double().flatten()
        got = gr[torch.from_numpy(gz[f"g:{n}:pos"]).to(dev)].float().cpu()
        ref = torch.from_numpy(gz[f"g:{n}:val"])
        mref, nref = float(gz[f"g:{n}:maxabs"]), float(gz[f"g:{n}:norm"])
        if _zero_grad_param(n):
            # mathematically zero (a softmax-row shift): rounding noise on both sides. The reference's
            # own bf16 run leaves ~2e-5 x gmax of it (norm, fixture gb:); fp16's column sums of the
            # key gradients carry somewhat more
            assert mref < 1e-6 * gmax, (n, mref)
            lim = {"fp32": 1e-5, "autocast": 2e-4, "autocast16": 5e-4}[mode]
            assert float(gr.abs().max()) <= lim * gmax, n
            zero += 1
            continue
        nrm = float(gr.norm())
        if mode == "fp32":
            assert float((got - ref).abs().max()) <= 2e-3 * mref, (n, float((got - ref).abs().max()), mref)
            assert abs(nrm - nref) <= 1e-3 * nref, (n, nrm, nref)
        else:
            c_ref, r_ref = _ref_drift(gz, n)
            assert abs(nrm - nref) <= max(5e-2, abs(r_ref - 1) + 2e-2) * nref, (n, nrm, nref, r_ref)
            cos = F.cosine_similarity(got.reshape(1, -1), ref.reshape(1, -1)).item()
            lim = min(0.99 if mref > 1e-3 * gmax else 0.95, c_ref - 0.02)
            assert cos >= lim, (n, cos, c_ref)
        checked += 1
    assert checked + zero == len(names) == 276 and zero == 24
    assert any(n.startswith("lm_head.") for n in names)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grad_stats(named_grads, gz):
    out = {}
    for n in (str(x) for x in gz["names"]):
        g = named_grads[ALIAS.get(n, n)].double().flatten()
        out[n] = (float(g.norm()), g[torch.from_numpy(gz[f"g:{n}:pos"]).to(g.device)].cpu().numpy())
    return out


@pytest.mark.parametrize("mode", ["fp32", "autocast"])
def test_c4_pretrain_dp_world2(dev, tmp_path, mode):
    gz = np.load(FIX)
    port = _free_port()
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    # fresh interpreters (the ranks never inherit this process's device state)
    procs = [subprocess.Popen([sys.executable, "-m", "tests._pretrain_dp_worker", str(tmp_path), mode], cwd=ROOT,
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(2)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=400)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]

    # one process on the whole batch: total loss, and the contrastive part alone (no MLM inputs)
    m = build_model(dev)
    batch = {k: v.to(dev) for k, v in fixture_inputs(gz).items()}
    with _ctx(mode):
        full = m(**batch)
    full.loss.backward()
    g_full = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    with _ctx(mode):
        cl = m(**{k: v for k, v in batch.items() if not k.startswith("mlm_")})
    cl.loss.backward()
    expect = {}
    for n, g in g_full.items():
        p = dict(m.named_parameters())[n]
        expect[n] = g - 0.5 * p.grad if p.grad is not None else g
    exp_stats = _grad_stats(expect, gz)

    rank_losses = [float(r["loss"]) for r in ranks]
    for r in ranks:
        assert int(r["correct"]) == int(full.cl_correct_num)
        assert int(r["collectives"]) == int(r["nbuckets"]) >= 2
    tol = 1e-5 if mode == "fp32" else 1e-2
    assert abs(np.mean(rank_losses) - float(full.loss)) <= tol * abs(float(full.loss)), (rank_losses, float(full.loss))
    gmax = max(float(np.abs(v[1]).max()) for v in exp_stats.values())
    nmax = max(v[0] for v in exp_stats.values())
    for n, (nrm_e, sl_e) in exp_stats.items():
        nrm0, sl0 = float(ranks[0][f"{n}:norm"]), ranks[0][f"{n}:val"]
        nrm1, sl1 = float(ranks[1][f"{n}:norm"]), ranks[1][f"{n}:val"]
        assert nrm0 == nrm1 and np.array_equal(sl0, sl1), n  # the all-reduced average is the same on both ranks
        if _zero_grad_param(n):  # mathematically zero: rounding noise on both sides
            assert nrm0 <= 1e-4 * nmax and nrm_e <= 1e-4 * nmax, n
            continue
        if mode == "fp32":
            assert abs(nrm0 - nrm_e) <= 1e-4 * nrm_e, (n, nrm0, nrm_e)
            assert float(np.abs(sl0 - sl_e).max()) <= 1e-4 * max(float(np.abs(sl_e).max()), 1e-12) + 1e-9, n
        else:
            assert abs(nrm0 - nrm_e) <= 3e-2 * nrm_e, (n, nrm0, nrm_e)
            if float(np.abs(sl_e).max()) > 1e-3 * gmax:
                cos = float(np.dot(sl0, sl_e) / (np.linalg.norm(sl0) * np.linalg.norm(sl_e) + 1e-30))
                assert cos >= 0.99, (n, cos)
