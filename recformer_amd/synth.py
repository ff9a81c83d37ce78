"""Synthetic Recformer workloads shared by tests, bench and fixtures.

Configs: C1 = 2L/d128/H2 (the reference's CPU-runnable case); BASE = longformer-base
dims (12L/768d/H12/hd64, ffn 3072, maxpos 4098, eps 1e-5) with window 64.
"""
from __future__ import annotations

import torch

C1 = dict(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
          intermediate_size=512, max_position_embeddings=514, layer_norm_eps=1e-5,
          attention_window=[64, 64], max_item_embeddings=51, token_type_size=4,
          pad_token_id=1, bos_token_id=0, hidden_dropout_prob=0.1,
          attention_probs_dropout_prob=0.1, temp=0.05)

BASE = dict(vocab_size=50265, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
            intermediate_size=3072, max_position_embeddings=4098, layer_norm_eps=1e-5,
            attention_window=[64] * 12, max_item_embeddings=51, token_type_size=4,
            pad_token_id=1, bos_token_id=0, hidden_dropout_prob=0.1,
            attention_probs_dropout_prob=0.1, temp=0.05)


def synth_batch(B, L, vocab, seed, lens=None, item_len=5, extra_globals=()):
    """Token ids U[3,vocab) with <s>=0 at t=0; type 0 at t=0 else U{1,2}; item-pos
    1+(t-1)//item_len clamped to 50; global one-hot at 0. `lens` pads rows as the
    reference tokenizer does (tokenization.py:134-138: id 1, item-pos 50, type 3)."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(3, vocab, (B, L), generator=g)
    ids[:, 0] = 0
    tt = torch.randint(1, 3, (B, L), generator=g)
    tt[:, 0] = 0
    ip = torch.clamp(1 + (torch.arange(L) - 1) // item_len, max=50).expand(B, L).clone()
    ip[:, 0] = 0
    am = torch.ones(B, L, dtype=torch.long)
    gm = torch.zeros(B, L, dtype=torch.long)
    gm[:, 0] = 1
    if lens is not None:
        for b, n in enumerate(lens):
            am[b, n:] = 0
            ids[b, n:] = 1
            ip[b, n:] = 50
            tt[b, n:] = 3
    for b, p in extra_globals:
        gm[b, p] = 1
    return dict(input_ids=ids, attention_mask=am, global_attention_mask=gm, token_type_ids=tt,
                item_position_ids=ip)
