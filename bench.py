"""bench.py — user-sequences/sec (encode + score) at 12L/768d, seq_len 1024, window 64.

One step = RecformerForSeqRec.forward (no labels) over one batch of B synthetic user
sequences already resident in HBM: fused prologue + embedding/LN, 12 Longformer layers
(MFMA GEMMs, banded local + global attention, LayerNorms), CLS pooling and cosine scores
against a 10,000-item catalog (BASELINE.json configs[1]). fp32 parameters
under torch.autocast(bf16) (the reference's mixed precision): bf16 GEMM / attention operands,
fp32 accumulation, fp32 residual stream; random-init weights of the longformer-base shape.

N GPUs (torchrun, one process per GPU): every rank encodes its own B sequences (weak
scaling, no data-path collective: user sequences are independent); the
catalog is replicated. value = all ranks' sequences / max-over-ranks time.

Prints ONE JSON line on rank 0 (plus the roofline of the dominant kernel measured with
HIP events inside the timed region, the attention-kernel HBM roofline, and — rank 0 at
N=1 only — the CPU baseline: the fp32 CPU restatement of the reference timed on a bounded
sample on this host's cores).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "user-sequences/sec (encode+score) at 12L/768d seq_len=1024, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=160, help="timed steps (default ~2.2 s of sustained load)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64, help="user sequences per GPU per step")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--catalog", type=int, default=10000)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16",
                    help="autocast dtype of the GEMM / attention operands (fp32 parameters)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0,
                    help="target CPU work for the baseline samples, split over the thread counts (0 disables)")
    ap.add_argument("--cpu-threads", type=str, default="all,omp",
                    help="thread counts for the CPU baseline: 'all' = every CPU this process may use "
                         "(affinity capped by the cgroup CPU quota), 'omp' = OMP_NUM_THREADS, or integers")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--full-last-layer", action="store_true",
                    help="every row through the last layer (default: the CLS rows only, which is all the "
                         "scores read; recformer_amd.models._cls_last_layer)")
    ap.add_argument("--no-full-leg", action="store_true",
                    help="skip the second timed leg with every row through the last layer (reported next to "
                         "the headline value so kernel progress stays comparable round over round)")
    ap.add_argument("--timing-steps", type=int, default=20,
                    help="steps of the separate HIP-event-instrumented pass (per-kernel times)")
    ap.add_argument("--batch-sweep", type=str, default="1,16,128",
                    help="SURVEY §8d batch sweep: per-GPU batch sizes timed eager and as a replayed HIP graph "
                         "(recformer_amd.graphs.GraphedForward) after the headline legs ('' disables; N=1 only)")
    return ap.parse_args()


def batch_sweep(model, cfg, L, sizes, amp, dev):
    """Per-batch-size latency and throughput of the same encode + score step, eager (one host read of the
    global-token count per forward) and replayed from a captured HIP graph (inputs copied into the
    graph's static tensors, no host read). B = 16 is the reference drivers' evaluation batch
    (finetune.py:185 -> eval, finetune.py:66-96)."""
    from recformer_amd.graphs import GraphedForward
    from recformer_amd.synth import synth_batch
    rows = []
    for Bs in sizes:
        bb = {k: v.to(dev) for k, v in synth_batch(Bs, L, cfg.vocab_size, seed=200 + Bs, item_len=21).items()}
        n = max(10, min(200, 2048 // Bs))
        with torch.autocast("cuda", dtype=amp):
            for _ in range(3):
                model(**bb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                model(**bb)
            torch.cuda.synchronize()
            eager = (time.perf_counter() - t0) / n
            g = GraphedForward(model, bb, check=False)
            for _ in range(3):
                g(**bb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                g(**bb)
            torch.cuda.synchronize()
            graphed = (time.perf_counter() - t0) / n
            del g
        torch.cuda.empty_cache()
        rows.append({"batch": Bs, "steps": n, "eager_ms": round(eager * 1e3, 3),
                     "eager_seq_s": round(Bs / eager, 1), "graphed_ms": round(graphed * 1e3, 3),
                     "graphed_seq_s": round(Bs / graphed, 1)})
    return rows


def gemm_flops_per_seq(L, d, ffn, layers, gmax=1, fold=True):
    # per layer: fused q,k,v (3 d x d over all L tokens; + k_g, v_g when the global
    # projections are not folded) + q_g (d x d on G rows) + out-proj (d x d) + FFN (2 d x ffn);
    # 2 flops per MAC. The global fold's own work (u = Wkg^T qg, P.H, Wvg GEMV) is excluded.
    per_layer = 2 * L * d * ((3 if fold else 5) * d) + 2 * gmax * d * d + 2 * L * d * d + 2 * 2 * L * d * ffn
    return per_layer * layers


def step_flops_per_seq(L, d, ffn, layers, catalog, w=64, gmax=1, cls_last=True):
    """Algorithmic flops per sequence of the step as it runs (SURVEY §8d counting: the GEMMs with the
    global projections folded, the exact band attention 4*d*sum|keys_i| + 4*G*L*d per layer with
    |keys_i| = w + 1 + G, the catalog scoring 2*N*d). cls_last: the last layer on the CLS rows only
    (models._cls_last_layer, what RecformerForSeqRec runs when every CLS is global) — its q_g projection
    on the G global rows, the global rows' attention over all L keys, and out-proj + FFN on the one CLS
    row; its local q|k|v projection, band attention and L-row GEMMs are not run."""
    full = layers - 1 if cls_last else layers
    gemm = gemm_flops_per_seq(L, d, ffn, full, gmax)
    attn = full * (4 * d * L * (w + 1 + gmax) + 4 * gmax * L * d)
    if cls_last:
        gemm += 2 * gmax * d * d + 2 * d * d + 2 * 2 * d * ffn
        attn += 4 * gmax * L * d
    score = 2 * catalog * d
    return {"gemm": gemm, "attn": attn, "score": score, "total": gemm + attn + score}


def e2e_floor_us(L, d, ffn, layers, catalog, w=64, gmax=1, cls_last=True):
    """End-to-end MFMA bound per sequence of the step as it runs, at 2.5 PF dense bf16:
    176.5 GFLOP -> 70.6 us/seq with every row through the last layer, 161.8 GFLOP -> 64.7 us/seq with
    the CLS-only last layer."""
    f = step_flops_per_seq(L, d, ffn, layers, catalog, w, gmax, cls_last)["total"]
    return f / (BF16_PEAK_TFLOPS * 1e12) * 1e6


def committed_profile(B, L, layers):
    """Per-kernel-tag rows of the newest committed rocprofv3 summary of this exact workload
    (profiles/r*/bench_pmc_summary.json, tools/profile_bench.sh: kernel-trace durations, HBM bytes
    from the FETCH_SIZE / WRITE_SIZE passes, MFMA-busy from the SQ_VALU_MFMA_BUSY_CYCLES pass), or {}."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "bench_pmc_summary.json")),
                       reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("config") == {"batch": B, "seq_len": L, "layers": layers}:
            return doc["tags"], os.path.relpath(path, ROOT)
    return {}, None


def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "cpu"


def _cpu_quota():
    """CPUs this process may use: the affinity set, capped by the cgroup's CPU quota (cgroup v2
    cpu.max or v1 cfs_quota_us). On the GPU box os.cpu_count() shows the whole machine while the
    quota is the per-GPU share; threads beyond the quota only contend."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        avail = max(1, min(avail, math.ceil(quota)))
    return avail


def _thread_counts(spec):
    avail = _cpu_quota()
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if tok == "all":
            n = avail
        elif tok == "omp":
            n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, avail)
        else:
            n = int(tok)
        n = max(1, min(n, avail))
        if n not in out:
            out.append(n)
    return out, avail


def _cpu_calibration():
    """The newest committed calibration of the restatement against the real reference (within
    ±15%; oracle/calibrate_cpu.py, run in the build container, where the reference exists), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "cpu_calibration.json")), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
            return {"port_over_reference": doc["port_over_reference"], "within_15pct": doc["within_15pct"],
                    "threads": doc["threads"], "file": os.path.relpath(path, ROOT)}
        except (OSError, ValueError, KeyError):
            continue
    return None


def cpu_baseline(sd_cpu, cfg, items_cpu, L, target_s, spec):
    """Time the CPU restatement of the reference (oracle/restatement.py: fp32, the reference's
    algorithm incl. broadcast cosine scoring) on a bounded sample of the same workload, at each
    requested thread count (all of the host's CPUs; also the box's per-GPU share).
    The fastest is reported as the baseline; every count's rate is listed."""
    from oracle import restatement as R  # cpu_baseline leg only
    from recformer_amd.synth import synth_batch

    counts, avail = _thread_counts(spec)
    if len(counts) > 1:
        # thread counts past the CPUs really available (an unreported quota) only contend: probe
        # each with a small fp32 GEMM and drop those slower than the best probe
        x = torch.randn(512, 768)
        w = torch.randn(768, 3072)
        probe = {}
        for T in counts:
            torch.set_num_threads(T)
            torch.mm(x, w)
            t0 = time.perf_counter()
            for _ in range(3):
                torch.mm(x, w)
            probe[T] = time.perf_counter() - t0
        best_p = min(probe.values())
        skipped = {str(T): f"GEMM probe {probe[T] / best_p:.1f}x slower" for T in counts if probe[T] > 1.5 * best_p}
        counts = [T for T in counts if probe[T] <= 1.5 * best_p]
    else:
        skipped = {}
    per = target_s / len(counts)
    b1 = synth_batch(1, L, cfg.vocab_size, seed=1234, item_len=21)
    bs = synth_batch(64, L, cfg.vocab_size, seed=4321, item_len=21)
    by = {}
    samples = {}
    for T in counts:
        torch.set_num_threads(T)
        t0 = time.perf_counter()
        _, z = R.model_forward(sd_cpu, cfg, **b1)  # warm + size the sample
        R.cosine_scores(z, items_cpu, cfg.temp)
        one = time.perf_counter() - t0
        n = max(1, min(64, int(per / max(one, 1e-3))))
        t0 = time.perf_counter()
        for i in range(n):
            _, z = R.model_forward(sd_cpu, cfg, **{k: v[i:i + 1] for k, v in bs.items()})
            R.cosine_scores(z, items_cpu, cfg.temp)
        by[T] = n / (time.perf_counter() - t0)
        samples[T] = n
    best = max(by, key=by.get)
    return {"value": by[best], "unit": "user-seq/s", "cores": best, "kind": "port",
            "calibration": _cpu_calibration(),
            "by_threads": {str(t): round(v, 3) for t, v in by.items()}, "skipped_threads": skipped,
            "sample": f"{samples[best]} sequences x L={L} (B=1 each) encode+score vs {items_cpu.shape[0]} items, "
                      f"fp32 oracle/restatement.py, {best} threads (fastest of {counts}) on {_cpu_model_name()} "
                      f"(os.cpu_count()={os.cpu_count()}; {avail} usable: affinity capped by the cgroup CPU quota)"}


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N ranks (one process per GPU) under torch.distributed.run
    from this GPU-free parent and exit with its status (the parent never touches the device)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # More ranks than devices (e.g. --gpus 2 on a one-GPU box, tools/gpu/dist_rehearsal.sh): the
    # ranks share the devices and the control collectives run on gloo (RCCL needs one rank per
    # device). Production runs use nccl (RCCL), one rank per GPU.
    ndev = torch.cuda.device_count()  # does not initialise the device
    rehearsal = os.environ.get("RF_BENCH_REHEARSAL") == "1" or (world > 1 and ndev < world)
    if rehearsal:
        local = local % max(ndev, 1)
    if world > 1:
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    coll_dev = None if rehearsal else dev

    from recformer_amd import RecformerConfig, RecformerForSeqRec, dp, models, ops
    from recformer_amd.synth import BASE, synth_batch
    if args.full_last_layer:
        models.PRUNE_LAST_LAYER = False

    L, B = args.seq_len, args.batch
    cfg = RecformerConfig(**dict(BASE, num_hidden_layers=args.layers,
                                 attention_window=[64] * args.layers, item_num=args.catalog))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg).eval()
    items = torch.randn(args.catalog, cfg.hidden_size) * 0.5
    model.init_item_embedding(items)
    want_cpu = (rank == 0 and world == 1 and args.cpu_baseline_seconds > 0)
    sd_cpu = {k: v.clone() for k, v in model.longformer.state_dict().items()} if want_cpu else None
    # the reference's mixed-precision mode: fp32 parameters under torch.autocast (the mode whose
    # parity is pinned at the north star's 1e-2, tests/test_gpu_model.py); the kernels read cached
    # 16-bit copies of the weights, so the step does the same work as with 16-bit parameters
    model = model.to(dev)
    amp = {"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]

    batch = synth_batch(B, L, cfg.vocab_size, seed=100 + rank, item_len=21)
    batch = {k: v.to(dev) for k, v in batch.items()}

    def step():
        with torch.autocast("cuda", dtype=amp):
            return model(**batch)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            scores = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # second leg: the same step with every row through the last layer (the kernels' work of a
        # 12-full-layer encode; comparable with rounds before the CLS-only last layer)
        elapsed_full = None
        if not args.full_last_layer and not args.no_full_leg:
            models.PRUNE_LAST_LAYER = False
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed_full = time.perf_counter() - t1
            models.PRUNE_LAST_LAYER = True
            for _ in range(3):
                step()
            torch.cuda.synchronize()
        # per-kernel breakdown from a separate instrumented pass (HIP events around every
        # launch), so the event records never sit inside the timed steps
        kt, inst_steps, inst_s = {}, 0, 0.0
        if not args.no_kernel_timing:
            inst_steps = max(1, args.timing_steps)
            ops.enable_timing(True)
            ti = time.perf_counter()
            for _ in range(inst_steps):
                step()
            torch.cuda.synchronize()
            inst_s = time.perf_counter() - ti
            kt = ops.timing_results()
            ops.enable_timing(False)
        sweep = None
        if args.batch_sweep and world == 1:
            sweep = batch_sweep(model, cfg, L, [int(x) for x in args.batch_sweep.split(",") if x.strip()], amp, dev)
    assert scores.shape == (B, args.catalog)

    tmax = dp.max_over_ranks(elapsed, device=coll_dev)
    total_seqs = B * world * args.steps
    value = total_seqs / tmax
    tmax_full = dp.max_over_ranks(elapsed_full, device=coll_dev) if elapsed_full is not None else None

    out = None
    if rank == 0:
        d, ffn = cfg.hidden_size, cfg.intermediate_size
        roofline = None
        attn_roof = None
        kernels = {}
        prof, prof_src = committed_profile(B, L, args.layers)
        if kt:
            for k, v in kt.items():
                kernels[k] = {"launches": len(v), "avg_us": 1e3 * sum(v) / len(v),
                              "median_us": 1e3 * sorted(v)[len(v) // 2],
                              "share_of_step": sum(v) / (inst_s * 1e3) if inst_s else None}
            gemms = {k: v for k, v in kt.items() if k.startswith("gemm_")}
            dom = max(gemms, key=lambda k: sum(gemms[k])) if gemms else None
            if dom:
                Mrows = B * L
                nqkv = 3 if getattr(cfg, "global_attention_fold", True) else 5
                nflops = {"gemm_qkv": 2 * Mrows * d * nqkv * d, "gemm_out": 2 * Mrows * d * d,
                          "gemm_ffn1": 2 * Mrows * d * ffn, "gemm_ffn2": 2 * Mrows * ffn * d}[dom]
                avg_s = sum(gemms[dom]) / len(gemms[dom]) / 1e3
                ach = nflops / avg_s / 1e12
                pr = prof.get(dom, {})
                p_us = pr.get("median_us") or pr.get("avg_us")
                roofline = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1),
                            "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(ach / BF16_PEAK_TFLOPS, 4), "traffic": pr.get("hbm_bytes"),
                            "traffic_unit": "HBM bytes per launch (PMC)",
                            "algorithmic_per_launch": f"{nflops / 1e9:.2f} GFLOP (2*M*N*K, M=B*L={Mrows})",
                            "avg_us_live": round(avg_s * 1e6, 2),
                            "profile_us": p_us, "profile_frac": (round(nflops / (p_us * 1e-6) / 1e12 / BF16_PEAK_TFLOPS, 4)
                                                                 if p_us else None),
                            "mfma_busy": pr.get("mfma_busy"), "profile_source": prof_src}
            if "band_attn" in kt:
                v = kt["band_attn"]
                avg_s = sum(v) / len(v) / 1e3
                nbytes = 8 * B * L * d  # read Q, K, V + write O, bf16
                gbs = nbytes / avg_s / 1e9
                attn_roof = {"kernel": "band_attn", "bound": "hbm", "achieved": round(gbs, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "traffic": prof.get("band_attn", {}).get("hbm_bytes"),
                             "traffic_unit": "HBM bytes per launch (PMC)", "profile_source": prof_src,
                             "profile_us": prof.get("band_attn", {}).get("median_us"),
                             "algorithmic_per_launch": f"{nbytes / 1e6:.1f} MB (8*B*L*d bytes)"}
        cls_last = not args.full_last_layer
        fl = step_flops_per_seq(L, d, ffn, args.layers, args.catalog, cls_last=cls_last)
        floor = e2e_floor_us(L, d, ffn, args.layers, args.catalog, cls_last=cls_last)
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "user-seq/s",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (seeded ids/types/item-pos, random-init weights of the 12L/768d shape)",
            "config": {"workload": "C2: RecformerForSeqRec encode+score, 12L/768d/H12, seq_len 1024, "
                                   "window 64, CLS global, 10k-item cosine scoring",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": L,
                       "catalog": args.catalog, "layers": args.layers,
                       "last_layer": ("all rows" if args.full_last_layer else
                                      "CLS rows only (the scores read nothing else; same scores)"),
                       "parallelism": f"dp{world} (independent sequence shards, replicated catalog)",
                       **({"ranks_share_devices": ndev} if rehearsal else {})},
            "roofline": roofline,
            "attention_roofline": attn_roof,
            # the algorithmic flops of the step as it runs (GEMMs + band attention + scoring)
            "model_tflops": round(value / world * fl["total"] / 1e12, 1),
            "gflop_per_seq": {k: round(v / 1e9, 3) for k, v in fl.items()},
            # end to end against the MFMA bound of the algorithm as run
            "e2e_roofline": {"bound": "mfma", "us_per_seq_floor": round(floor, 2),
                             "frac": round(value / world * floor * 1e-6, 4),
                             "note": "per-GPU seq/s x the MFMA-bound us per sequence of the step as run"},
        }
        if tmax_full is not None:
            v_full = total_seqs / tmax_full
            floor_full = e2e_floor_us(L, d, ffn, args.layers, args.catalog, cls_last=False)
            out["value_full_last_layer"] = round(v_full, 2)
            out["full_last_layer"] = {"ms_per_step": round(1e3 * tmax_full / args.steps, 3), "steps": args.steps,
                                      "e2e_frac": round(v_full / world * floor_full * 1e-6, 4),
                                      "us_per_seq_floor": round(floor_full, 2),
                                      "note": "same process, same batch, every row through the last layer "
                                              "(models.PRUNE_LAST_LAYER=False)"}
        if sweep:
            out["batch_sweep"] = {"rows": sweep, "note": "same process after the timed legs, same model and mode; "
                                  "eager = RecformerForSeqRec.forward per batch, graphed = GraphedForward replay "
                                  "(inputs copied in); B=64 is the headline"}
        out.update({
            "kernels": kernels,
            "kernels_pass": ({"steps": inst_steps, "ms_per_step": round(1e3 * inst_s / inst_steps, 3),
                              "note": "separate HIP-event-instrumented steps after the timed ones"}
                             if inst_steps else None),
        })
        if want_cpu:
            items_cpu = items.float()
            out["cpu_baseline"] = cpu_baseline(sd_cpu, cfg, items_cpu, L, args.cpu_baseline_seconds,
                                               args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
