"""Kernel sequence of a rocprofv3 kernel trace (csv), short names, durations and gaps:
    python tools/trace_seq.py TRACE.csv [first] [count]"""
import csv
import sys

KEYS = ["k_score_rank", "k_rank_w32", "k_topk_merge", "k_topk_dense", "k_rank_reduce", "row_inv_norm", "FillFunctor",
        "partition_kernel", "block_reduce", "copyBuffer", "fillBuffer", "transform_kernel", "init_lookback",
        "label_score", "direct_copy", "normal", "float16_copy"]


def short(n):
    for k in KEYS:
        if k in n:
            return k + ("<1>" if "Li1E" in n else "<0>" if "Li0E" in n else "<2>" if "Li2E" in n else "")
    return n[:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    a = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    prev = None
    for i, r in enumerate(rows[a:a + n], a):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        prev = e
        print(f"{i:5d} {short(r['Kernel_Name']):20s} {(e - s) / 1e3:9.1f} us  gap {gap:8.1f}")


if __name__ == "__main__":
    main()
