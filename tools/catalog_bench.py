"""C5-style full-catalog retrieval (BASELINE configs[4]) on one GPU: encode a synthetic item
catalog (<s> + 32 tokens per item, L=33 padded to 64, batches of `--batch` items), then score Q
user vectors against the whole catalog (cosine / temp on the MFMA GEMM, fp32 scores resident in
HBM) and compute the Ranker metrics (rf_rank_accum). Under torchrun each rank encodes its shard
of the catalog and the embeddings are all-gathered (recformer_amd.dp.gather_rows).

    python tools/catalog_bench.py [--items 262144] [--queries 4096] [--batch 4096]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from recformer_amd import Ranker, RecformerConfig, RecformerModel, dp, ops  # noqa: E402
from recformer_amd.ranker import rank_catalog  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=262144)
    ap.add_argument("--queries", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    dev = torch.device("cuda")
    cfg = RecformerConfig(**BASE)
    torch.manual_seed(0)
    model = RecformerModel(cfg).eval().to(dev).to(torch.bfloat16)
    lo, hi = dp.shard_range(a.items, rank, world)
    # one synthetic item batch re-used (token content does not change the work)
    tmpl = {k: v.to(dev) for k, v in synth_batch(a.batch, 33, cfg.vocab_size, seed=5, item_len=32).items()}
    embs = []
    with torch.no_grad():
        model(**{k: v[:64] for k, v in tmpl.items()})  # warm up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(lo, hi, a.batch):
            n = min(a.batch, hi - s)
            embs.append(model(**{k: v[:n] for k, v in tmpl.items()}).pooler_output.to(torch.bfloat16))
        torch.cuda.synchronize()
        t_enc = time.perf_counter() - t0
        local = torch.cat(embs, 0)
        table = dp.gather_rows(local, a.items) if world > 1 else local
        q = torch.randn(a.queries, cfg.hidden_size, device=dev).to(torch.bfloat16)
        labels = torch.randint(0, a.items, (a.queries,), device=dev)
        t_parts = []
        for _ in range(2):  # the first pass also pays the score buffer's allocation
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rn = ops.row_inv_norm(table)
            scores = ops.cos_scores(q, table, 1.0 / cfg.temp, items_rnorm=rn)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            metrics = Ranker([10, 50])(scores, labels)
            torch.cuda.synchronize()
            t_parts.append((t1 - t0, time.perf_counter() - t1))
            del scores
        t_score = sum(t_parts[-1])
        # the same metrics block by block (ranker.rank_catalog: no (B, N) score matrix)
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            metrics_blk = rank_catalog(q, table, labels, [10, 50], cfg.temp)
            torch.cuda.synchronize()
            t_blk = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"workload": "C5-style retrieval: encode catalog (L=33->64) + score/rank queries",
                          "items": a.items, "queries": a.queries, "gpus": world,
                          "encode_s": round(t_enc, 3), "items_per_s": round((hi - lo) * world / t_enc, 1),
                          "score_rank_ms": round(1e3 * t_score, 2),
                          "score_ms": round(1e3 * t_parts[-1][0], 2), "rank_ms": round(1e3 * t_parts[-1][1], 2),
                          "first_pass_ms": round(1e3 * sum(t_parts[0]), 2),
                          "blockwise_score_rank_ms": round(1e3 * t_blk, 2),
                          "blockwise_metrics_equal": metrics_blk[:-1] == metrics[:-1],
                          "score_tflops": round(2 * a.queries * a.items * cfg.hidden_size / t_score / 1e12, 1),
                          "scores_gb": round(a.queries * a.items * 4 / 2**30, 2), "metrics": [round(m, 4) for m in metrics]}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
