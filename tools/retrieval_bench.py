"""C5 scoring throughput (BASELINE configs[4]): Q queries against a catalog shard with the fused
score + rank + top-50 kernels (recformer_amd.ranker.shard_rank), one GPU.

    python tools/retrieval_bench.py [--queries 4096] [--items 125000,1000000] [--dtype fp16]

Prints per shard size: ms per call, query-item pairs/s, TFLOP/s of the score GEMM (2*Q*N*d) and
its fraction of the 2.5 PF dense fp16/bf16 MFMA peak; the counts-only mode (rank_catalog) too. Each mode
runs on the kernel family the product path picks for it (ranker._rank_family: the 16x16x32 rank loop
with a top-k, the 32x32x16 one for counts only) unless RF_KNOBS pins rank_w32."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import contextlib  # noqa: E402

from recformer_amd.ranker import CatalogShard, _rank_family, label_scores, shard_rank  # noqa: E402


@contextlib.contextmanager
def _knob_ctx(name, value):
    from recformer_amd import _lib
    old = _lib.set_knob(name, value)
    try:
        yield
    finally:
        _lib.set_knob(name, old)


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=4096)
    ap.add_argument("--items", type=str, default="125000,1000000")
    ap.add_argument("--dtype", type=str, default="fp16")
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--growth", type=str, default="",
                    help="comma list of ranker.TOPK_GROWTH values to time the top-k mode at (A/B); default: the "
                         "module's")
    ap.add_argument("--family", type=str, default="", help="A/B: 'w16,w32' times the top-k mode on both families")
    args = ap.parse_args()
    import recformer_amd.ranker as RK
    from recformer_amd import _lib
    pinned = False
    for kv in filter(None, os.environ.get("RF_KNOBS", "").split(",")):  # e.g. RF_KNOBS=rank_w32=1
        k, v = kv.split("=")
        _lib.set_knob(k, int(v))
        pinned = pinned or k == "rank_w32"
    family = (lambda topk: contextlib.nullcontext()) if pinned else _rank_family
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Q, d = args.queries, 768
    q = torch.randn(Q, d, device=dev, generator=g).to(dt)
    for N in (int(x) for x in args.items.split(",")):
        items = torch.randn(N, d, device=dev, generator=g).to(dt)
        labels = torch.randint(0, N, (Q,), device=dev, generator=g)
        shard = CatalogShard(items)
        with family(True):  # label scores from the same family as the ranking (exact strict counts)
            sl = label_scores(q, shard, labels, 0.05)
            t_top = timeit(lambda: shard_rank(q, shard, sl, 0.05, k=args.k))
            ref = shard_rank(q, shard, sl, 0.05, k=args.k)
        # A/B of the top-k plan (the same result required): growth factors x kernel families
        for fam in [f for f in args.family.split(",") if f] or ([""] if args.growth else []):
            for gr in [x for x in args.growth.split(",") if x] or [str(RK.TOPK_GROWTH)]:
                old_g = RK.TOPK_GROWTH
                RK.TOPK_GROWTH = int(gr)
                ctx = (contextlib.nullcontext() if not fam else
                       _knob_ctx("rank_w32", 1 if fam == "w32" else 0))
                with ctx:
                    slf = label_scores(q, shard, labels, 0.05)
                    t = timeit(lambda: shard_rank(q, shard, slf, 0.05, k=args.k))
                    r = shard_rank(q, shard, slf, 0.05, k=args.k)
                RK.TOPK_GROWTH = old_g
                same = bool(torch.equal(r["topi"], ref["topi"]) and torch.equal(r["gt"], ref["gt"]))
                print(json.dumps({"items": N, "ab": f"growth={gr} family={fam or 'default'}", "ms": round(t * 1e3, 3),
                                  "frac_of_2.5PF": round(2.0 * Q * N * d / t / 2.5e15, 3), "same_result": same}),
                      flush=True)
        with family(False):
            sl = label_scores(q, shard, labels, 0.05)
            t_cnt = timeit(lambda: shard_rank(q, shard, sl, 0.05, k=0))
        fl = 2.0 * Q * N * d
        for name, t in (("rank+top%d" % args.k, t_top), ("rank only", t_cnt)):
            print(json.dumps({"items": N, "queries": Q, "dtype": args.dtype, "mode": name, "ms": round(t * 1e3, 3),
                              "pairs_per_s": round(Q * N / t / 1e9, 2), "tflops": round(fl / t / 1e12, 1),
                              "frac_of_2.5PF": round(fl / t / 2.5e15, 3)}), flush=True)
        del items, shard


if __name__ == "__main__":
    main()
