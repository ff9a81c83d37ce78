"""CPU-baseline calibration: the restatement that bench.py times on the GPU box's host
cores as `cpu_baseline` must run within ±15% of the REAL reference on the same cores. Build container
only (the reference is loaded through oracle/ref_harness.py; it does not exist on the GPU box).

ORACLE / TEST INFRASTRUCTURE — never imported by the product package.

Workload: bench.py's cpu_baseline sample — C2 encode + score, B = 1 sequence of L = 1024 tokens
(12L/768d, window 64, CLS global), cosine scores against a 10,000-item catalog, fp32, both sides on the
same inputs and the same hash-initialised weights, the same torch thread count. The reference path is
RecformerForSeqRec.forward (recformer/models.py:547-599: longformer encode, pooler, similarity_score
over the whole item table, models.py:539-545); the restatement path is oracle/restatement.py
model_forward + cosine_scores, exactly what bench.cpu_baseline runs.

    python oracle/calibrate_cpu.py [--threads 8] [--seqs 6] [--out profiles/r05/cpu_calibration.json]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from oracle import restatement as R  # noqa: E402
from oracle.ref_harness import load_reference_models, make_reference_config  # noqa: E402
from recformer_amd.hashinit import hash_init_, hash_tensor  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--seqs", type=int, default=6)
    ap.add_argument("--catalog", type=int, default=10000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "cpu_calibration.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    M = load_reference_models()
    ref = M.RecformerForSeqRec(make_reference_config(item_num=a.catalog, **BASE)).eval()
    hash_init_(ref.longformer, seed=2)
    items = hash_tensor("catalog", (a.catalog, 768), "weight", seed=3, std=1.0)
    ref.init_item_embedding(items)
    sd = {k: v.clone() for k, v in ref.longformer.state_dict().items()}
    cfg = ref.config
    bs = synth_batch(a.seqs + 1, 1024, BASE["vocab_size"], seed=4321, item_len=21)
    one = [{k: v[i:i + 1] for k, v in bs.items()} for i in range(a.seqs + 1)]

    def run_ref(b):
        return ref(**b)

    def run_port(b):
        _, z = R.model_forward(sd, cfg, **b)
        return R.cosine_scores(z, items, cfg.temp)

    res = {}
    with torch.no_grad():
        # agreement on the first sequence (the calibration compares the same computation)
        s_ref, s_port = run_ref(one[0]), run_port(one[0])
        diff = float((s_ref - s_port).abs().max())
        for name, fn in (("reference", run_ref), ("port", run_port), ("reference_again", run_ref),
                         ("port_again", run_port)):
            fn(one[0])  # warm
            t0 = time.perf_counter()
            for b in one[1:]:
                fn(b)
            res[name] = a.seqs / (time.perf_counter() - t0)
    r_ref = 0.5 * (res["reference"] + res["reference_again"])
    r_port = 0.5 * (res["port"] + res["port_again"])
    doc = {"workload": "C2 encode+score, B=1, L=1024, 12L/768d, window 64, CLS global, "
                       f"{a.catalog}-item cosine scores, fp32",
           "threads": a.threads, "cpu": _cpu_model(), "os_cpu_count": os.cpu_count(), "seqs_per_leg": a.seqs,
           "reference_seq_per_s": round(r_ref, 3), "port_seq_per_s": round(r_port, 3),
           "legs_seq_per_s": {k: round(v, 3) for k, v in res.items()},
           "port_over_reference": round(r_port / r_ref, 4),
           "within_15pct": abs(r_port / r_ref - 1.0) <= 0.15,
           "scores_max_abs_diff": diff,
           "reference": "recformer/models.py RecformerForSeqRec.forward via oracle/ref_harness.py "
                        "(transformers 5.15 + 3 shims)",
           "port": "oracle/restatement.py model_forward + cosine_scores (bench.py cpu_baseline)",
           "torch": torch.__version__}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
