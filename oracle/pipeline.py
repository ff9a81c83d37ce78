"""CPU restatement of the reference's input pipeline for pre-tokenized items — ORACLE.

ORACLE / TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does). Restates
RecformerTokenizer.encode(items, encode_item=False) and .padding (recformer/tokenization.py)
and the collators' glue (collator.py:245-385) in plain Python lists, line by line. Pinned
against the reference itself by tests/golden/pipeline.npz (oracle/gen_golden_pipeline.py runs
the real tokenization.py).
"""
from __future__ import annotations


def encode(items, max_items, max_tokens, bos_id):
    """tokenization.py:64-105 with encode_item=False; items = [[input_ids, token_type_ids], ...]
    in past...present order."""
    items = items[::-1]                                  # :70
    items = items[:max_items - 1]                        # :71
    input_ids, item_position_ids, token_type_ids = [bos_id], [0], [0]   # :73-75
    for item_idx, (ids, tts) in enumerate(items):       # :77-91
        input_ids += list(ids)
        token_type_ids += list(tts)
        item_position_ids += [item_idx + 1] * len(ids)
    input_ids = input_ids[:max_tokens]                   # :93-95
    item_position_ids = item_position_ids[:max_tokens]
    token_type_ids = token_type_ids[:max_tokens]
    attention_mask = [1] * len(input_ids)                # :97-99
    global_attention_mask = [0] * len(input_ids)
    global_attention_mask[0] = 1
    return {"input_ids": input_ids, "item_position_ids": item_position_ids, "token_type_ids": token_type_ids,
            "attention_mask": attention_mask, "global_attention_mask": global_attention_mask}


def padding(batch, pad_to_max, max_items, max_tokens, pad_id):
    """tokenization.py:108-152."""
    L = max_tokens if pad_to_max else max(len(x["input_ids"]) for x in batch)
    out = {k: [] for k in batch[0]}
    for x in batch:
        n = L - len(x["input_ids"])
        out["input_ids"].append(x["input_ids"] + [pad_id] * n)
        out["item_position_ids"].append(x["item_position_ids"] + [max_items - 1] * n)
        out["token_type_ids"].append(x["token_type_ids"] + [3] * n)
        out["attention_mask"].append(x["attention_mask"] + [0] * n)
        out["global_attention_mask"].append(x["global_attention_mask"] + [0] * n)
    return out


def collate(tokenized_items, seqs, max_items, max_tokens, bos_id, pad_id, pad_to_max=False):
    """collator.py extract_features -> encode_features -> padding (:292-313, :358-385)."""
    feats = [[list(tokenized_items[i]) for i in s] for s in seqs]
    return padding([encode(f, max_items, max_tokens, bos_id) for f in feats], pad_to_max, max_items,
                   max_tokens, pad_id)
