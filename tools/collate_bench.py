"""Host batch-building throughput: the C++ builder (recformer_amd.data.collate) vs the
reference-style Python path (oracle/pipeline.py restates tokenization.py encode/padding +
torch.LongTensor, collator.py:292-313) on C3-shaped batches (50 items x 32 tokens -> 1024).

    python tools/collate_bench.py [B]
"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import pipeline as P  # noqa: E402  (the timed Python baseline)
from recformer_amd import data as D  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    rng = random.Random(0)
    items = {i: [[rng.randint(3, 50000) for _ in range(32)], [1, 1] + [2] * 30] for i in range(10000)}
    store = D.ItemStore(items)
    batches = [[[rng.randrange(10000) for _ in range(50)] for _ in range(B)] for _ in range(20)]
    t0 = time.perf_counter()
    for bt in batches[:5]:
        ref = P.collate(items, bt, 51, 1024, 0, 1)
        {k: torch.LongTensor(v) for k, v in ref.items()}
    py = 5 * B / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for bt in batches:
        D.collate(store, bt, 51, 1024, 0, 1)
    cpp = len(batches) * B / (time.perf_counter() - t0)
    print(f"B={B}: python (reference-style) {py:,.0f} seq/s | C++ builder {cpp:,.0f} seq/s (one core)")


if __name__ == "__main__":
    main()
