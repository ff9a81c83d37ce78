"""Host input pipeline for pre-tokenized items, backed by the C++
batch builder librecformer_host.so (include/recformer_host.h).

Drop-ins for the reference's pipeline pieces:
  * ItemStore            — the `tokenized_items` dict {item: [input_ids, token_type_ids]}
                           (finetune.py:239-245) flattened to CSR arrays, built once;
  * collate()            — RecformerTokenizer.encode(items, encode_item=False) + padding()
                           + torch.LongTensor (tokenization.py:64-152) for a whole batch in
                           one C++ call, written into (optionally pinned) int64 tensors;
  * FinetuneDataCollatorWithPadding / EvalDataCollatorWithPadding (collator.py:245-385):
                           same constructor fields, same __call__ contract and outputs, the
                           same Python `random` draws for the training target;
  * RecformerTokenizer   — the reference's tokenizer class (tokenization.py:4-159): the BPE
                           item encoding is transformers' LongformerTokenizer as in the
                           reference; batch_encode of pre-tokenized items goes through C++.

The collators accept any tokenizer exposing `.config` (max_item_embeddings, max_token_num),
`.bos_token_id` and `.pad_token_id` — the reference's own RecformerTokenizer included.
"""
from __future__ import annotations

import ctypes
import operator
import os
import random
from ctypes import c_int, c_int64, c_void_p
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librecformer_host.so")
_HLIB: Optional[ctypes.CDLL] = None

KEYS = ("input_ids", "item_position_ids", "token_type_ids", "attention_mask", "global_attention_mask")


class RecformerHostError(RuntimeError):
    pass


def load_host(path: str = HOST_LIB_PATH) -> ctypes.CDLL:
    global _HLIB
    if _HLIB is not None:
        return _HLIB
    if not os.path.isfile(path):
        raise RecformerHostError(f"librecformer_host.so not found at {path}: build with make -C recformer_amd/csrc")
    lib = ctypes.CDLL(path)
    P = c_void_p
    lib.rf_host_last_error.restype = ctypes.c_char_p
    lib.rf_host_last_error.argtypes = []
    lib.rf_collate_lengths.restype = c_int
    lib.rf_collate_lengths.argtypes = [c_int, P, P, c_int64, P, c_int, c_int, P]
    lib.rf_collate_fill.restype = c_int
    lib.rf_collate_fill.argtypes = [c_int, c_int, P, P, c_int64, P, P, P, c_int, c_int, c_int, c_int,
                                    P, P, P, P, P]
    _HLIB = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RecformerHostError(f"{what} failed: {load_host().rf_host_last_error().decode(errors='replace')}")


def _ptr(a) -> int:
    return a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr()


class ItemStore:
    """CSR form of {item: [input_ids, token_type_ids]}. Items are addressed by their dict key
    (any hashable); keys 0..n-1 in order map to themselves without a dict lookup."""

    def __init__(self, tokenized_items: Dict):
        keys = list(tokenized_items.keys())
        self.n = len(keys)
        self._dense = keys == list(range(self.n))
        self.index = None if self._dense else {k: i for i, k in enumerate(keys)}
        lens = np.zeros(self.n + 1, dtype=np.int64)
        ids, types = [], []
        for i, k in enumerate(keys):
            a, t = tokenized_items[k]
            if len(a) != len(t):
                raise ValueError(f"item {k!r}: input_ids and token_type_ids differ in length")
            lens[i + 1] = len(a)
            ids.append(np.asarray(a, dtype=np.int32))
            types.append(np.asarray(t, dtype=np.int32))
        self.item_off = np.cumsum(lens)
        self.tok_ids = np.concatenate(ids) if ids else np.zeros(0, np.int32)
        self.tok_types = np.concatenate(types) if types else np.zeros(0, np.int32)

    def indices(self, seq: Sequence) -> List[int]:
        if not self._dense:
            return [self.index[k] for k in seq]
        try:
            return [operator.index(k) for k in seq]  # range-checked by the C++ builder
        except TypeError as e:
            raise KeyError(f"item keys of this store are 0..{self.n - 1}") from e


def collate(store: ItemStore, seqs: Sequence[Sequence], max_items: int, max_tokens: int, bos_id: int,
            pad_id: int, pad_to_max: bool = False, pin_memory: bool = False) -> Dict[str, torch.Tensor]:
    """encode(seq, encode_item=False) for every item sequence (past ... present) + padding, as
    five (B, L) int64 tensors; L = max encoded length, or max_tokens with pad_to_max."""
    lib = load_host()
    B = len(seqs)
    flat = [store.indices(s) for s in seqs]
    seq_off = np.zeros(B + 1, dtype=np.int64)
    seq_off[1:] = np.cumsum([len(s) for s in flat])
    seq_items = np.fromiter((i for s in flat for i in s), dtype=np.int64, count=int(seq_off[-1]))
    lens = np.zeros(max(B, 1), dtype=np.int32)
    _check(lib.rf_collate_lengths(B, _ptr(seq_off), _ptr(seq_items), store.n, _ptr(store.item_off),
                                  max_items, max_tokens, _ptr(lens)), "rf_collate_lengths")
    L = max_tokens if pad_to_max else (int(lens[:B].max()) if B else 1)
    out = {k: torch.empty(B, L, dtype=torch.int64, pin_memory=pin_memory) for k in KEYS}
    _check(lib.rf_collate_fill(B, L, _ptr(seq_off), _ptr(seq_items), store.n, _ptr(store.item_off),
                               _ptr(store.tok_ids), _ptr(store.tok_types), max_items, max_tokens, bos_id,
                               pad_id, *(_ptr(out[k]) for k in KEYS)), "rf_collate_fill")
    return out


def _cfg_limits(tokenizer):
    c = tokenizer.config
    return c.max_item_embeddings, c.max_token_num, tokenizer.bos_token_id, tokenizer.pad_token_id


@dataclass
class FinetuneDataCollatorWithPadding:
    """collator.py:245-313: per sequence a random target position (Python `random`, as the
    reference), the items before it as the input, the target item as the label."""
    tokenizer: object
    tokenized_items: Dict
    pin_memory: bool = False

    def __post_init__(self):
        self.store = ItemStore(self.tokenized_items)

    def sample_train_data(self, batch_item_ids):
        batch_item_seq, labels = [], []
        for item_ids in batch_item_ids:
            item_ids = item_ids["items"]
            n = len(item_ids)
            target_pos = random.randint(min(n, 0), n - 1)
            batch_item_seq.append(item_ids[:target_pos])
            labels.append(item_ids[target_pos])
        return batch_item_seq, labels

    def __call__(self, batch_item_ids):
        seqs, labels = self.sample_train_data(batch_item_ids)
        mi, mt, bos, pad = _cfg_limits(self.tokenizer)
        batch = collate(self.store, seqs, mi, mt, bos, pad, pin_memory=self.pin_memory)
        batch["labels"] = torch.tensor(labels, dtype=torch.int64)
        return batch


@dataclass
class EvalDataCollatorWithPadding:
    """collator.py:316-385: (batch, labels) for {'items': [...], 'label': item}."""
    tokenizer: object
    tokenized_items: Dict
    pin_memory: bool = False

    def __post_init__(self):
        self.store = ItemStore(self.tokenized_items)

    def __call__(self, batch_data):
        seqs = [d["items"] for d in batch_data]
        labels = torch.tensor([d["label"] for d in batch_data], dtype=torch.int64)
        mi, mt, bos, pad = _cfg_limits(self.tokenizer)
        return collate(self.store, seqs, mi, mt, bos, pad, pin_memory=self.pin_memory), labels


def _longformer_tokenizer_base():
    try:
        from transformers import LongformerTokenizer
        return LongformerTokenizer
    except Exception:  # transformers absent: the pre-tokenized paths still work
        return object


class RecformerTokenizer(_longformer_tokenizer_base()):
    """tokenization.py:4-159 — the same methods and outputs. Text -> BPE ids is transformers'
    LongformerTokenizer (as in the reference); sequences of pre-tokenized items are encoded and
    padded by the C++ batch builder when a batch is requested as tensors."""

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, config=None):
        cls.config = config  # tokenization.py:7 keeps the config on the class
        return super().from_pretrained(pretrained_model_name_or_path)

    def __call__(self, items, pad_to_max=False, return_tensor=False):
        if len(items) > 0 and isinstance(items[0], list):
            inputs = self.batch_encode(items, pad_to_max=pad_to_max)
        else:
            inputs = self.encode(items)
        if return_tensor:
            for k, v in inputs.items():
                inputs[k] = torch.LongTensor(v)
        return inputs

    def item_tokenize(self, text):
        return self.convert_tokens_to_ids(self.tokenize(text))

    def encode_item(self, item):
        input_ids, token_type_ids = [], []
        for attr_name, attr_value in list(item.items())[:self.config.max_attr_num]:
            name_tokens = self.item_tokenize(attr_name)
            value_tokens = self.item_tokenize(attr_value)
            input_ids += (name_tokens + value_tokens)[:self.config.max_attr_length]
            token_type_ids += ([1] * len(name_tokens) + [2] * len(value_tokens))[:self.config.max_attr_length]
        return input_ids, token_type_ids

    def encode(self, items, encode_item=True):
        feats = [self.encode_item(it) if encode_item else it for it in items[::-1][:self.config.max_item_embeddings - 1]]
        store = ItemStore({i: f for i, f in enumerate(feats)})
        b = collate(store, [list(range(len(feats)))[::-1]], self.config.max_item_embeddings,
                    self.config.max_token_num, self.bos_token_id, self.pad_token_id)
        return {k: v[0].tolist() for k, v in b.items()}

    def padding(self, item_batch, pad_to_max):
        L = self.config.max_token_num if pad_to_max else max(len(x["input_ids"]) for x in item_batch)
        fill = {"input_ids": self.pad_token_id, "item_position_ids": self.config.max_item_embeddings - 1,
                "token_type_ids": 3, "attention_mask": 0, "global_attention_mask": 0}
        out = {k: [] for k in KEYS}
        for x in item_batch:
            n = L - len(x["input_ids"])
            for k in KEYS:
                x[k] += [fill[k]] * n  # in place, as the reference (tokenization.py:134-138)
                out[k].append(x[k])
        return out

    def batch_encode(self, item_batch, encode_item=True, pad_to_max=False):
        return self.padding([self.encode(items, encode_item) for items in item_batch], pad_to_max)

    def batch_encode_tensors(self, item_batch, encode_item=True, pad_to_max=False, pin_memory=False):
        """batch_encode + torch.LongTensor in one C++ pass (the collators' path)."""
        seqs, feats = [], {}
        for items in item_batch:
            seq = []
            for it in items:
                feats[len(feats)] = self.encode_item(it) if encode_item else it
                seq.append(len(feats) - 1)
            seqs.append(seq)
        return collate(ItemStore(feats), seqs, self.config.max_item_embeddings, self.config.max_token_num,
                       self.bos_token_id, self.pad_token_id, pad_to_max=pad_to_max, pin_memory=pin_memory)
