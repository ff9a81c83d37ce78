"""Golden vectors for the host input pipeline from the REAL reference tokenizer (test infra).

Loads /root/reference/recformer/tokenization.py by file path (it imports only torch and
transformers), with a subclass that sets bos/pad ids and the config instead of loading a BPE
vocabulary (encode(encode_item=False) and padding() never touch the vocabulary). Writes
tests/golden/pipeline.npz: a random pre-tokenized item store (CSR), item sequences (CSR) and the
reference's batch_encode outputs for pad_to_max False / True.

    python oracle/gen_golden_pipeline.py
"""
import importlib.util
import os
import sys
from types import SimpleNamespace

import numpy as np

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    spec = importlib.util.spec_from_file_location("_ref_tok", "/root/reference/recformer/tokenization.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)

    class StubTok(mod.RecformerTokenizer):
        bos_token_id = 0
        pad_token_id = 1

        def __init__(self):  # no vocabulary: only the pre-tokenized paths are exercised
            pass

    cfg = SimpleNamespace(max_item_embeddings=51, max_token_num=1024, max_attr_num=12, max_attr_length=32)
    StubTok.config = cfg
    tok = StubTok()
    rng = np.random.default_rng(7)
    n_items = 300
    lens = rng.integers(0, 41, n_items)
    lens[:3] = (0, 1, 40)
    items = {}
    for i in range(n_items):
        ids = rng.integers(3, 50265, lens[i]).tolist()
        tts = [1] * min(2, lens[i]) + [2] * max(0, lens[i] - 2)
        items[i] = [ids, tts]
    out = {}
    batches = {"a": [0, 1, 5, 49, 50, 51, 80, 20, 33, 12, 0, 64], "b": [0, 3, 1, 7]}
    for name, seq_lens in batches.items():
        seqs = [rng.integers(0, n_items, n).tolist() for n in seq_lens]
        for pad_to_max in (False, True):
            feats = [[items[i] for i in s] for s in seqs]
            res = tok.batch_encode([[list(map(list, f)) for f in fs] for fs in feats], encode_item=False,
                                   pad_to_max=pad_to_max)
            for k, v in res.items():
                out[f"{name}_{k}_{'max' if pad_to_max else 'dyn'}"] = np.asarray(v, dtype=np.int64)
        out[f"{name}_seq_off"] = np.concatenate([[0], np.cumsum(seq_lens)]).astype(np.int64)
        out[f"{name}_seq_items"] = np.concatenate([np.asarray(s, np.int64) for s in seqs] + [np.zeros(0, np.int64)])
    item_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    tok_ids = np.concatenate([np.asarray(items[i][0], np.int64) for i in range(n_items)])
    tok_types = np.concatenate([np.asarray(items[i][1], np.int64) for i in range(n_items)])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "pipeline.npz"), item_off=item_off, tok_ids=tok_ids,
                        tok_types=tok_types, limits=np.array([51, 1024, 0, 1], np.int64), **out)
    print("wrote tests/golden/pipeline.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
