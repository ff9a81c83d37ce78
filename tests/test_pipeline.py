"""Host input pipeline: the C++ batch builder (librecformer_host.so,
include/recformer_host.h) against the pipeline oracle (oracle/pipeline.py) and the golden
vectors of the REAL reference tokenizer (tests/golden/pipeline.npz, oracle/gen_golden_pipeline.py).
Bit-exact integer outputs. CPU only."""
import os
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import pipeline as P
from recformer_amd import data as D

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pipeline.npz")


def _store_from_golden(g):
    off, ids, tts = g["item_off"], g["tok_ids"], g["tok_types"]
    return {i: [ids[off[i]:off[i + 1]].tolist(), tts[off[i]:off[i + 1]].tolist()] for i in range(len(off) - 1)}


@pytest.mark.parametrize("batch", ["a", "b"])
@pytest.mark.parametrize("pad_to_max", [False, True])
def test_collate_matches_reference_golden(batch, pad_to_max):
    g = np.load(GOLD)
    mi, mt, bos, pad = (int(x) for x in g["limits"])
    items = _store_from_golden(g)
    so, si = g[f"{batch}_seq_off"], g[f"{batch}_seq_items"]
    seqs = [si[so[b]:so[b + 1]].tolist() for b in range(len(so) - 1)]
    out = D.collate(D.ItemStore(items), seqs, mi, mt, bos, pad, pad_to_max=pad_to_max)
    ref = P.collate(items, seqs, mi, mt, bos, pad, pad_to_max=pad_to_max)
    sfx = "max" if pad_to_max else "dyn"
    for k in D.KEYS:
        gold = g[f"{batch}_{k}_{sfx}"]
        assert np.array_equal(np.asarray(ref[k]), gold), f"oracle vs reference golden: {k}"
        assert out[k].dtype == torch.int64 and np.array_equal(out[k].numpy(), gold), k


def test_collate_random_vs_oracle():
    rng = random.Random(3)
    items = {}
    for i in range(500):
        n = rng.randint(0, 60)
        items[f"item{i}"] = [[rng.randint(3, 50000) for _ in range(n)], [rng.choice((1, 2)) for _ in range(n)]]
    keys = list(items)
    store = D.ItemStore(items)
    for trial in range(20):
        mi, mt = rng.choice([(51, 1024), (5, 64), (2, 16), (51, 33)])
        seqs = [[rng.choice(keys) for _ in range(rng.randint(0, 70))] for _ in range(rng.randint(1, 9))]
        for pad_to_max in (False, True):
            out = D.collate(store, seqs, mi, mt, 0, 1, pad_to_max=pad_to_max)
            ref = P.collate(items, seqs, mi, mt, 0, 1, pad_to_max=pad_to_max)
            for k in D.KEYS:
                assert np.array_equal(out[k].numpy(), np.asarray(ref[k])), (trial, k)


def test_collators_mirror_reference_contract():
    tok = SimpleNamespace(config=SimpleNamespace(max_item_embeddings=51, max_token_num=1024), bos_token_id=0,
                          pad_token_id=1)
    items = {i: [[10 + i] * (1 + i % 7), [1] + [2] * (i % 7)] for i in range(100)}
    data = [{"items": [3, 5, 7, 11, 13]}, {"items": [2]}, {"items": list(range(60))}]
    random.seed(11)
    batch = D.FinetuneDataCollatorWithPadding(tok, items)(data)
    random.seed(11)  # the reference draws the same targets from Python's random (collator.py:282-284)
    seqs, labels = [], []
    for d in data:
        t = random.randint(0, len(d["items"]) - 1)
        seqs.append(d["items"][:t])
        labels.append(d["items"][t])
    ref = P.collate(items, seqs, 51, 1024, 0, 1)
    assert batch["labels"].tolist() == labels
    for k in D.KEYS:
        assert np.array_equal(batch[k].numpy(), np.asarray(ref[k]))
    ev = [{"items": [1, 2, 3], "label": 4}, {"items": [], "label": 9}]
    b2, lab = D.EvalDataCollatorWithPadding(tok, items)(ev)
    assert lab.tolist() == [4, 9]
    ref = P.collate(items, [[1, 2, 3], []], 51, 1024, 0, 1)
    for k in D.KEYS:
        assert np.array_equal(b2[k].numpy(), np.asarray(ref[k]))


def test_collate_errors_are_reported():
    store = D.ItemStore({0: [[5], [1]]})
    with pytest.raises(KeyError):
        D.collate(store, [["missing"]], 51, 1024, 0, 1)
    lib = D.load_host()
    off = np.array([0, 1], np.int64)
    bad = np.array([7], np.int64)
    lens = np.zeros(1, np.int32)
    rc = lib.rf_collate_lengths(1, off.ctypes.data, bad.ctypes.data, 1, store.item_off.ctypes.data, 51, 1024,
                                lens.ctypes.data)
    assert rc != 0 and b"out of range" in lib.rf_host_last_error()


def test_tokenizer_pretokenized_paths_match_oracle():
    """recformer_amd.RecformerTokenizer's encode / padding / batch_encode (encode_item=False)
    without a BPE vocabulary (the pre-tokenized paths never touch it)."""
    class Tok(D.RecformerTokenizer):
        bos_token_id = 0
        pad_token_id = 1

        def __init__(self):
            pass

    Tok.config = SimpleNamespace(max_item_embeddings=6, max_token_num=40, max_attr_num=12, max_attr_length=32)
    tok = Tok()
    rng = random.Random(5)
    seqs = [[[[rng.randint(3, 99) for _ in range(n)], [2] * n] for n in (rng.randint(0, 9) for _ in range(k))]
            for k in (0, 3, 9)]
    ref = P.padding([P.encode(s, 6, 40, 0) for s in seqs], False, 6, 40, 1)
    got = tok.batch_encode(seqs, encode_item=False)
    assert got == ref
    t = tok.batch_encode_tensors(seqs, encode_item=False)
    for k in D.KEYS:
        assert t[k].tolist() == ref[k]
    assert tok.encode(seqs[1], encode_item=False) == P.encode(seqs[1], 6, 40, 0)
