"""Generate tests/golden/ranker.npz from the REAL reference Ranker (build container only).

ORACLE / TEST INFRASTRUCTURE. Loads /root/reference/utils.py by file path (it imports only
json / torch / torch.nn) and runs `Ranker(ks)(scores, labels)` (utils.py:76-108) on fixed score
matrices built to stress the strict-rank contract: exact ties with the label's score, rows
whose label sits in the last ragged columns, a row count that is not a multiple of 16, entries
at or below -MAX_VAL (utils.py:5: excluded from valid_length), and a cosine/temp-shaped case.
The fixture stores inputs and the reference's outputs (data only, no reference source).

    python oracle/gen_golden_ranker.py
"""
from __future__ import annotations

import importlib.util
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_UTILS = "/root/reference/utils.py"
KS = [1, 5, 10, 20, 50]


def load_ranker():
    spec = importlib.util.spec_from_file_location("_ref_utils", REF_UTILS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Ranker


def cases():
    g = torch.Generator().manual_seed(7)
    out = {}
    # (a) B=37 rows x N=1000 columns, scores quantised to 1/8 so ties are frequent; labels forced
    # into the last partial 16-column group for a third of the rows
    B, N = 37, 1000
    s = torch.round(torch.randn(B, N, generator=g) * 16) / 8
    lab = torch.randint(0, N, (B,), generator=g)
    lab[::3] = N - 1 - torch.randint(0, 8, (len(lab[::3]),), generator=g)
    out["ties"] = (s, lab)
    # (b) some entries masked to -MAX_VAL (the reference's valid_length excludes them) and one
    # row whose label score is the row maximum, one where it is the minimum
    s2 = torch.randn(20, 333, generator=g) * 3
    s2[:, 300:] = -1e4
    s2[3, :250] = -2e4
    lab2 = torch.randint(0, 300, (20,), generator=g)
    s2[5, lab2[5]] = 50.0
    s2[6, lab2[6]] = -50.0
    out["masked"] = (s2, lab2)
    # (c) the model's score distribution: cosine / 0.05 (|s| <= 20), B=64 x N=1531
    q = torch.nn.functional.normalize(torch.randn(64, 32, generator=g), dim=-1)
    e = torch.nn.functional.normalize(torch.randn(1531, 32, generator=g), dim=-1)
    s3 = (q @ e.t()) / 0.05
    lab3 = torch.randint(0, 1531, (64,), generator=g)
    out["cosine"] = (s3, lab3)
    return out


def main():
    Ranker = load_ranker()
    r = Ranker(KS)
    arrays = {"ks": np.asarray(KS)}
    for name, (s, lab) in cases().items():
        res = r(s.clone(), lab.clone())
        arrays[f"{name}_scores"] = s.numpy().astype(np.float32)
        arrays[f"{name}_labels"] = lab.numpy()
        arrays[f"{name}_metrics"] = np.asarray(res, dtype=np.float64)
        # the per-row strict ranks behind the means (same expressions as utils.py:92-94)
        pred = s[torch.arange(s.size(0)), lab].unsqueeze(-1)
        arrays[f"{name}_rank"] = (pred < s).sum(-1).numpy()
        arrays[f"{name}_valid"] = (s > -1e4).sum(-1).numpy()
    path = os.path.join(ROOT, "tests", "golden", "ranker.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
