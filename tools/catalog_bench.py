"""C5 full-catalog retrieval (BASELINE configs[4]): encode a synthetic item catalog sharded over
the ranks (<s> + 32 tokens per item, batches of `--batch`
items, fp16 autocast by default; L=33 runs unpadded (Lp=33) through the short-sequence attention kernel unless
--pad64), keep each rank's embeddings as its CatalogShard (no gather of
the table), all-gather the Q query vectors, and rank them against the whole catalog with the
fused score + rank + top-50 kernels (recformer_amd.retrieve: per-shard counts and top-k,
all-reduce / all-gather across ranks). One rank per GPU under torchrun.

    python tools/catalog_bench.py [--items 1000000] [--queries 4096] [--batch 4096] [--dtype fp16]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from recformer_amd import CatalogShard, RecformerConfig, RecformerModel, dp, retrieve  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=1000000)
    ap.add_argument("--queries", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", choices=["fp16", "bf16"], default="fp16")
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--pad64", action="store_true", help="pad L=33 to the 64-token window (no short path)")
    ap.add_argument("--full-last-layer", action="store_true", help="A/B: every row through the last layer")
    a = ap.parse_args()
    if a.pad64:
        from recformer_amd import models
        models.SHORT_SEQ = False
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    dev = torch.device("cuda")
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    cfg = RecformerConfig(**BASE)
    torch.manual_seed(0)
    model = RecformerModel(cfg).eval().to(dev)
    lo, hi = dp.shard_range(a.items, rank, world)
    # one synthetic item batch re-used (token content does not change the work)
    tmpl = {k: v.to(dev) for k, v in synth_batch(a.batch, 33, cfg.vocab_size, seed=5, item_len=32).items()}
    embs = []
    with torch.no_grad(), torch.autocast("cuda", dtype=dt):
        model(**{k: v[:64] for k, v in tmpl.items()})  # warm up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(lo, hi, a.batch):
            n = min(a.batch, hi - s)
            # pooler_output only (finetune.py:38-63): the last layer runs on the CLS rows (models._cls_last_layer)
            embs.append(model(**{k: v[:n] for k, v in tmpl.items()}, _pooled_only=not a.full_last_layer)
                        .pooler_output.to(dt))
        torch.cuda.synchronize()
        t_enc = time.perf_counter() - t0
    shard = CatalogShard(torch.cat(embs, 0), base=lo)
    # the queries: each rank's share of the users' CLS vectors, all-gathered
    g = torch.Generator(device=dev).manual_seed(11)
    q_all = torch.randn(a.queries, cfg.hidden_size, device=dev, generator=g).to(dt)
    qa, qb = dp.shard_range(a.queries, rank, world)
    queries = dp.gather_rows(q_all[qa:qb].contiguous(), a.queries)
    labels = torch.randint(0, a.items, (a.queries,), device=dev, generator=g)
    times = []
    for _ in range(3):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        metrics, topv, topi = retrieve(queries, shard, labels, [10, 50], cfg.temp, k=a.k)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t_ret = dp.max_over_ranks(min(times), device=dev)
    t_enc = dp.max_over_ranks(t_enc, device=dev)
    if rank == 0:
        print(json.dumps({"workload": "C5 retrieval: encode a catalog shard per GPU (L=33->" + ("64" if a.pad64 else "33, unpadded") + "), fused score + rank + "
                                      f"top-{a.k} over the sharded catalog", "items": a.items, "queries": a.queries,
                          "gpus": world, "dtype": a.dtype, "encode_s": round(t_enc, 3),
                          "items_per_s": round(a.items / t_enc, 1), "retrieve_ms": round(1e3 * t_ret, 2),
                          "query_item_pairs_per_s": round(a.queries * a.items / t_ret / 1e9, 1),
                          "score_tflops_per_gpu": round(2 * a.queries * a.items * cfg.hidden_size / t_ret / world / 1e12, 1),
                          "metrics": [round(m, 4) for m in metrics], "top1_ids": topi[:4, 0].tolist()}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
