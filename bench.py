"""bench.py — user-sequences/sec (encode + score) at 12L/768d, seq_len 1024, window 64.

One step = RecformerForSeqRec.forward (no labels) over one batch of B synthetic user
sequences already resident in HBM: fused prologue + embedding/LN, 12 Longformer layers
(MFMA GEMMs, banded local + global attention, LayerNorms), CLS pooling and cosine scores
against a 10,000-item catalog (BASELINE.json configs[1]). bf16 weights
and activations, fp32 accumulation, random-init weights of the longformer-base shape.

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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="user sequences per GPU per step")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--catalog", type=int, default=10000)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="target CPU work for the baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-kernel-timing", action="store_true")
    return ap.parse_args()


def gemm_flops_per_seq(L, d, ffn, layers, gmax=1, fold=True):
    # per layer: fused q,k,v (3 d x d over all L tokens; + k_g, v_g when the global
    # projections are not folded) + q_g (d x d on G rows) + out-proj (d x d) + FFN (2 d x ffn);
    # 2 flops per MAC. The global fold's own work (u = Wkg^T qg, P.H, Wvg GEMV) is excluded.
    per_layer = 2 * L * d * ((3 if fold else 5) * d) + 2 * gmax * d * d + 2 * L * d * d + 2 * 2 * L * d * ffn
    return per_layer * layers


def pmc_traffic(B, L, layers):
    """Per-launch HBM bytes per kernel tag from the newest committed PMC profile of this exact
    workload (profiles/r*/bench_pmc_summary.json, tools/profile_bench.sh), or {}."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "bench_pmc_summary.json")),
                       reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("config") == {"batch": B, "seq_len": L, "layers": layers}:
            return {k: v.get("hbm_bytes") for k, v in doc["tags"].items()}, os.path.relpath(path, ROOT)
    return {}, None


def cpu_baseline(sd_cpu, cfg, items_cpu, L, target_s, threads):
    """Time the CPU restatement of the reference (oracle/restatement.py: fp32, the reference's
    algorithm incl. broadcast cosine scoring) on a bounded sample of the same workload."""
    from oracle import restatement as R  # cpu_baseline leg only
    from recformer_amd.synth import synth_batch

    torch.set_num_threads(threads)
    b1 = synth_batch(1, L, cfg.vocab_size, seed=1234, item_len=21)
    t0 = time.perf_counter()
    _, z = R.model_forward(sd_cpu, cfg, **b1)
    R.cosine_scores(z, items_cpu, cfg.temp)
    one = time.perf_counter() - t0
    n = max(1, min(64, int(target_s / max(one, 1e-3))))
    bs = synth_batch(n, L, cfg.vocab_size, seed=4321, item_len=21)
    t0 = time.perf_counter()
    for i in range(n):
        _, z = R.model_forward(sd_cpu, cfg, **{k: v[i:i + 1] for k, v in bs.items()})
        R.cosine_scores(z, items_cpu, cfg.temp)
    dt = time.perf_counter() - t0
    model_name = platform.processor() or "cpu"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n / dt, "unit": "user-seq/s", "cores": threads, "kind": "port",
            "sample": f"{n} sequences x L={L} (B=1 each) encode+score vs {items_cpu.shape[0]} items, "
                      f"fp32 oracle/restatement.py, {threads} threads on {model_name} "
                      f"(os.cpu_count()={os.cpu_count()})"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank control flow on a one-GPU box (tools/gpu/dist_rehearsal.sh): every
    # rank on cuda:0 with gloo collectives on host tensors. Production runs use nccl (RCCL).
    rehearsal = os.environ.get("RF_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    coll_dev = None if rehearsal else dev

    from recformer_amd import RecformerConfig, RecformerForSeqRec, dp, ops
    from recformer_amd.synth import BASE, synth_batch

    L, B = args.seq_len, args.batch
    cfg = RecformerConfig(**dict(BASE, num_hidden_layers=args.layers,
                                 attention_window=[64] * args.layers, item_num=args.catalog))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg).eval()
    items = torch.randn(args.catalog, cfg.hidden_size) * 0.5
    model.init_item_embedding(items)
    want_cpu = (rank == 0 and world == 1 and args.cpu_baseline_seconds > 0)
    sd_cpu = {k: v.clone() for k, v in model.longformer.state_dict().items()} if want_cpu else None
    model = model.to(dev).to(torch.bfloat16)

    batch = synth_batch(B, L, cfg.vocab_size, seed=100 + rank, item_len=21)
    batch = {k: v.to(dev) for k, v in batch.items()}

    def step():
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
        # per-kernel breakdown from a separate instrumented pass (HIP events around every
        # launch), so the event records never sit inside the timed steps
        kt, inst_steps, inst_s = {}, 0, 0.0
        if not args.no_kernel_timing:
            inst_steps = min(args.steps, 5)
            ops.enable_timing(True)
            ti = time.perf_counter()
            for _ in range(inst_steps):
                step()
            torch.cuda.synchronize()
            inst_s = time.perf_counter() - ti
            kt = ops.timing_results()
            ops.enable_timing(False)
    assert scores.shape == (B, args.catalog)

    tmax = dp.max_over_ranks(elapsed, device=coll_dev)
    total_seqs = B * world * args.steps
    value = total_seqs / tmax

    out = None
    if rank == 0:
        d, ffn = cfg.hidden_size, cfg.intermediate_size
        roofline = None
        attn_roof = None
        kernels = {}
        traffic, traffic_src = pmc_traffic(B, L, args.layers)
        if kt:
            for k, v in kt.items():
                kernels[k] = {"launches": len(v), "avg_us": 1e3 * sum(v) / len(v),
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
                roofline = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1),
                            "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(ach / BF16_PEAK_TFLOPS, 4), "traffic": traffic.get(dom),
                            "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                            "algorithmic_per_launch": f"{nflops / 1e9:.2f} GFLOP (2*M*N*K, M=B*L={Mrows})"}
            if "band_attn" in kt:
                v = kt["band_attn"]
                avg_s = sum(v) / len(v) / 1e3
                nbytes = 8 * B * L * d  # read Q, K, V + write O, bf16
                gbs = nbytes / avg_s / 1e9
                attn_roof = {"kernel": "band_attn", "bound": "hbm", "achieved": round(gbs, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "traffic": traffic.get("band_attn"),
                             "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                             "algorithmic_per_launch": f"{nbytes / 1e6:.1f} MB (8*B*L*d bytes)"}
        flops_seq = gemm_flops_per_seq(L, d, ffn, args.layers, fold=getattr(cfg, "global_attention_fold", True))
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "user-seq/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded ids/types/item-pos, random-init weights of the 12L/768d shape)",
            "config": {"workload": "C2: RecformerForSeqRec encode+score, 12L/768d/H12, seq_len 1024, "
                                   "window 64, CLS global, 10k-item cosine scoring",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": L,
                       "catalog": args.catalog, "layers": args.layers,
                       "parallelism": f"dp{world} (independent sequence shards, replicated catalog)"},
            "roofline": roofline,
            "attention_roofline": attn_roof,
            "model_tflops": round(value / world * flops_seq / 1e12, 1),
            "kernels": kernels,
            "kernels_pass": ({"steps": inst_steps, "ms_per_step": round(1e3 * inst_s / inst_steps, 3),
                              "note": "separate HIP-event-instrumented steps after the timed ones"}
                             if inst_steps else None),
        }
        if want_cpu:
            items_cpu = items.float()
            out["cpu_baseline"] = cpu_baseline(sd_cpu, cfg, items_cpu, L, args.cpu_baseline_seconds,
                                               min(args.cpu_threads, os.cpu_count() or 1))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
