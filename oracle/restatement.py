"""CPU restatement of the Recformer hot path (fp32 PyTorch) — the parity ORACLE.

ORACLE / TEST INFRASTRUCTURE ONLY. Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the checker /
the timed CPU baseline — never as the product path. The product (`recformer_amd`)
fails loudly when its HIP library is missing; it never routes through here.

Pinned against the reference itself: `oracle/gen_golden.py` runs the real
`recformer/models.py` (via `oracle/ref_harness.py`, transformers 5.15 + 3 shims) and
`tests/test_oracle_golden.py` checks this restatement against those fixtures.

Algorithm, with the reference file:line each step follows:
  * prologue: merge masks `models.py:262-272`, pad to a multiple of the window
    `models.py:210-260` (ids<-pad, item-pos<-pad_token_id (:244), type<-0, mask<-0)
  * embeddings `models.py:68-79, 108-138`: pos = cumsum(id!=pad)*(id!=pad)+pad;
    LN(Ew[id] + Ep[pos] + Et[tt] + Ei[ip])
  * per layer (transformers LongformerLayer, TF:1134-1172):
      - q,k,v projections, q /= sqrt(hd)                       TF:504-514
      - banded local scores |i-j| <= w/2 over valid non-global keys, plus one
        column per global key (local K)                        TF:519-569, 743-757
      - fp32 softmax; padded query rows -> 0                   TF:574-579
      - PV over band + global columns (local V)                TF:593-604, 928-962
      - global query rows overwritten by softmax(qg . kg) vg over all valid keys,
        kg/vg = key_global/value_global over ALL tokens        TF:964-1057, 612-629
      - a = LN(Wo ctx + bo + h); h = LN(W2 gelu(W1 a + b1) + b2 + a)   TF:1064-1131
  * crop padding TF:1229; 'cls' pooler models.py:160-171
  * cosine similarity / temp with broadcast (B,1,d) x (1,N,d) models.py:358-369, 539-545

The banded product is computed block-wise (64-query blocks against their 128-key
window), a different decomposition from transformers' overlapping-chunk einsum
but with a comparable ~2x flop overhead, so its CPU time is a fair stand-in for the
reference CPU path on the GPU box (where the reference cannot travel).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def prepare_inputs(input_ids, attention_mask, global_attention_mask, token_type_ids,
                   item_position_ids, window: int, pad_token_id: int = 1):
    """models.py:306-323 — merged mask {0,1,2}, padded to a multiple of `window`."""
    B, L = input_ids.shape
    if attention_mask is None:
        attention_mask = torch.ones_like(input_ids)
    if token_type_ids is None:
        token_type_ids = torch.zeros_like(input_ids)
    if global_attention_mask is not None:
        merged = attention_mask * (global_attention_mask + 1)
    else:
        merged = attention_mask
    pad = (window - L % window) % window
    if pad:
        input_ids = F.pad(input_ids, (0, pad), value=pad_token_id)
        item_position_ids = F.pad(item_position_ids, (0, pad), value=pad_token_id)
        merged = F.pad(merged, (0, pad), value=0)
        token_type_ids = F.pad(token_type_ids, (0, pad), value=0)
    return input_ids, merged, token_type_ids, item_position_ids, pad


def embeddings(sd: Dict[str, Tensor], p: str, ids, tt, ip, eps: float, pad_id: int = 1):
    m = (ids != pad_id).int()
    pos = (torch.cumsum(m, dim=1).type_as(m) * m).long() + pad_id
    x = (sd[p + "word_embeddings.weight"][ids] + sd[p + "position_embeddings.weight"][pos]
         + sd[p + "token_type_embeddings.weight"][tt] + sd[p + "item_position_embeddings.weight"][ip])
    return F.layer_norm(x, (x.shape[-1],), sd[p + "LayerNorm.weight"], sd[p + "LayerNorm.bias"], eps)


def _lin(x, sd, name):
    return F.linear(x, sd[name + ".weight"], sd[name + ".bias"])


def band_global_attention(q, k, v, merged, half_w: int, qg=None, kg=None, vg=None, head_mask=None,
                          probs_out=None):
    """q,k,v: (B,H,Lp,hd) (q pre-scaled). merged: (B,Lp) in {0,1,2}.

    Returns ctx (B,H,Lp,hd). If qg/kg/vg given, global rows are overwritten. `head_mask` (H,)
    multiplies the local and the global probabilities per head, as transformers 4.28.0's
    LongformerSelfAttention does with layer_head_mask (the version the reference pins; 5.15 has no
    head_mask, so this step is restated from 4.28's published code and is parity unpinned).
    `probs_out`, a list, receives (local, global) probabilities in the layout LongformerSelfAttention
    returns for output_attentions (TF:593-640): local (B,H,Lp,G+2w+1) = [global-key columns, band
    offsets -w..w], zero on padded and on global query rows (TF:626-629); global (B,H,G,Lp), the
    row of an empty global slot uniform (its all-min score row, TF:990-1000).
    """
    B, H, Lp, hd = q.shape
    W = 2 * half_w
    blk = W                        # queries per block
    nb = Lp // blk
    span = blk + 2 * half_w        # keys seen by a block
    valid = merged > 0
    glob = merged > 1
    local_key = valid & ~glob      # keys allowed inside the band

    kp = F.pad(k, (0, 0, half_w, half_w))
    vp = F.pad(v, (0, 0, half_w, half_w))
    kw = kp.unfold(2, span, blk).permute(0, 1, 2, 4, 3)        # (B,H,nb,span,hd)
    vw = vp.unfold(2, span, blk).permute(0, 1, 2, 4, 3)
    qb = q.reshape(B, H, nb, blk, hd)
    s_band = torch.matmul(qb, kw.transpose(-1, -2))             # (B,H,nb,blk,span)

    # allowed[b, n, i, j]: key position = n*blk + j - half_w, query = n*blk + i
    qi = torch.arange(blk).view(blk, 1)
    kj = torch.arange(span).view(1, span)
    rel = kj - half_w - qi                                       # key - query
    in_band = (rel.abs() <= half_w)
    kpos = (torch.arange(nb).view(nb, 1) * blk + torch.arange(span).view(1, span) - half_w)  # (nb,span)
    in_seq = (kpos >= 0) & (kpos < Lp)
    lk = F.pad(local_key, (half_w, half_w), value=False).unfold(1, span, blk)  # (B,nb,span)
    allowed = in_band.view(1, 1, blk, span) & (in_seq & True).view(1, nb, 1, span) & lk.view(B, nb, 1, span)
    s_band = s_band.masked_fill(~allowed.unsqueeze(1), float("-inf"))
    s_band = s_band.reshape(B, H, Lp, span)

    # global key columns (local K/V at global positions)
    gcount = glob.sum(1)
    G = int(gcount.max()) if B > 0 else 0
    if G > 0:
        gidx = torch.zeros(B, G, dtype=torch.long)
        gval = torch.zeros(B, G, dtype=torch.bool)
        for b in range(B):
            pos = torch.nonzero(glob[b], as_tuple=False).flatten()
            gidx[b, : pos.numel()] = pos
            gval[b, : pos.numel()] = True
        kgl = torch.gather(k, 2, gidx.view(B, 1, G, 1).expand(B, H, G, hd))
        vgl = torch.gather(v, 2, gidx.view(B, 1, G, 1).expand(B, H, G, hd))
        s_glob = torch.matmul(q, kgl.transpose(-1, -2))          # (B,H,Lp,G)
        s_glob = s_glob.masked_fill(~gval.view(B, 1, 1, G), float("-inf"))
        s = torch.cat([s_glob, s_band], dim=-1)
    else:
        s = s_band
    p = torch.softmax(s.float(), dim=-1)
    p = torch.where(valid.view(B, 1, Lp, 1), p, torch.zeros_like(p))
    if head_mask is not None:
        p = p * head_mask.float().view(1, H, 1, 1)
    if G > 0:
        p_glob, p_band = p[..., :G], p[..., G:]
        ctx = torch.matmul(p_glob, vgl)
    else:
        p_band = p
        ctx = torch.zeros_like(q)
    pb = p_band.reshape(B, H, nb, blk, span)
    ctx = ctx + torch.matmul(pb, vw).reshape(B, H, Lp, hd)
    if probs_out is not None:
        # band column c of query qi in its block is span column qi + c
        cols = (torch.arange(blk).view(blk, 1) + torch.arange(W + 1).view(1, W + 1))
        band = torch.gather(pb, 4, cols.view(1, 1, 1, blk, W + 1).expand(B, H, nb, blk, W + 1))
        local = band.reshape(B, H, Lp, W + 1)
        if G > 0:
            local = torch.cat([p_glob, local], dim=-1)
        local = local.masked_fill(glob.view(B, 1, Lp, 1), 0.0)

    if G > 0 and qg is not None:
        # qg: (B,H,G,hd) (pre-scaled) for the G global rows; kg, vg: (B,H,Lp,hd)
        sg = torch.matmul(qg, kg.transpose(-1, -2))              # (B,H,G,Lp)
        sg = sg.masked_fill(~valid.view(B, 1, 1, Lp), float("-inf"))
        pg = torch.softmax(sg.float(), dim=-1)
        if head_mask is not None:
            pg = pg * head_mask.float().view(1, H, 1, 1)
        og = torch.matmul(pg, vg)                                # (B,H,G,hd)
        if probs_out is not None:
            pgo = torch.where(gval.view(B, 1, G, 1), pg, torch.full_like(pg, 1.0 / Lp))
            if head_mask is not None:
                pgo = torch.where(gval.view(B, 1, G, 1), pgo, pgo * head_mask.float().view(1, H, 1, 1))
            probs_out.append((local, pgo))
        for b in range(B):
            n = int(gcount[b])
            if n:
                pos = gidx[b, :n]
                ctx[b, :, pos, :] = og[b, :, :n, :]
    elif probs_out is not None:
        probs_out.append((local, None))
    return ctx


def layer_forward(sd, p: str, h, merged, H: int, half_w: int, eps: float, head_mask=None, probs_out=None):
    B, Lp, D = h.shape
    hd = D // H
    a = p + "attention.self."

    def heads(x):
        return x.view(B, -1, H, hd).transpose(1, 2)

    q = heads(_lin(h, sd, a + "query") / math.sqrt(hd))
    k = heads(_lin(h, sd, a + "key"))
    v = heads(_lin(h, sd, a + "value"))
    glob = merged > 1
    qg = kg = vg = None
    if bool(glob.any()):
        G = int(glob.sum(1).max())
        hg = torch.zeros(B, G, D, dtype=h.dtype)
        for b in range(B):
            pos = torch.nonzero(glob[b], as_tuple=False).flatten()
            hg[b, : pos.numel()] = h[b, pos]
        qg = heads(_lin(hg, sd, a + "query_global") / math.sqrt(hd))
        kg = heads(_lin(h, sd, a + "key_global"))      # over ALL tokens, as TF:983-984
        vg = heads(_lin(h, sd, a + "value_global"))
    ctx = band_global_attention(q, k, v, merged, half_w, qg, kg, vg, head_mask, probs_out)
    ctx = ctx.transpose(1, 2).reshape(B, Lp, D)
    o = p + "attention.output."
    x = F.layer_norm(_lin(ctx, sd, o + "dense") + h, (D,), sd[o + "LayerNorm.weight"], sd[o + "LayerNorm.bias"], eps)
    f = F.gelu(_lin(x, sd, p + "intermediate.dense"))
    y = F.layer_norm(_lin(f, sd, p + "output.dense") + x, (D,), sd[p + "output.LayerNorm.weight"],
                     sd[p + "output.LayerNorm.bias"], eps)
    return y


def model_forward(sd: Dict[str, Tensor], cfg, input_ids, attention_mask=None, global_attention_mask=None,
                  token_type_ids=None, item_position_ids=None, prefix: str = "",
                  return_all_layers: bool = False, head_mask=None, probs_out=None):
    """RecformerModel.forward (models.py:274-356) -> (last_hidden_state, pooler_output); with
    `probs_out` (a list) also each layer's (local, global) attention probabilities over the padded
    length (band_global_attention)."""
    windows = cfg.window_per_layer() if hasattr(cfg, "window_per_layer") else (
        cfg.attention_window if isinstance(cfg.attention_window, list) else [cfg.attention_window] * cfg.num_hidden_layers)
    wmax = max(windows)
    L = input_ids.shape[1]
    ids, merged, tt, ip, pad = prepare_inputs(input_ids, attention_mask, global_attention_mask,
                                              token_type_ids, item_position_ids, wmax, cfg.pad_token_id)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in sd.items()}
    h = embeddings(sd, prefix + "embeddings.", ids, tt, ip, cfg.layer_norm_eps, cfg.pad_token_id)
    layers = [h]
    for i in range(cfg.num_hidden_layers):
        h = layer_forward(sd, f"{prefix}encoder.layer.{i}.", h, merged, cfg.num_attention_heads,
                          windows[i] // 2, cfg.layer_norm_eps, None if head_mask is None else head_mask[i],
                          probs_out)
        layers.append(h)
    h = h[:, :L]
    if cfg.pooler_type == "cls":
        pooled = h[:, 0]
    else:
        raise NotImplementedError(cfg.pooler_type)
    if return_all_layers:
        return h, pooled, [x[:, :L] for x in layers]
    return h, pooled


def cosine_scores(z: Tensor, items: Tensor, temp: float) -> Tensor:
    """Similarity.forward models.py:368-369 applied as in similarity_score :539-545
    (broadcast (B,1,d) x (1,N,d) or (B,C,d)), i.e. the reference's memory behaviour."""
    if items.dim() == 2:
        items = items.unsqueeze(0)
    return F.cosine_similarity(z.float().unsqueeze(1), items.float(), dim=-1) / temp


def seqrec_loss(scores: Tensor, labels: Tensor) -> Tensor:
    """models.py:587-597 — CrossEntropy over scores (full or sampled with target 0)."""
    return F.cross_entropy(scores, labels)


def lm_head_forward(sd: Dict[str, Tensor], x: Tensor, eps: float) -> Tensor:
    """LongformerLMHead.forward TF:1277-1285 (4.28 ties decoder.bias to bias): dense -> exact
    GELU -> LayerNorm -> decoder; sd holds the lm_head.* parameters without the prefix."""
    t = F.gelu(x @ sd["dense.weight"].t() + sd["dense.bias"])
    t = F.layer_norm(t, (t.shape[-1],), sd["layer_norm.weight"], sd["layer_norm.bias"], eps)
    return t @ sd["decoder.weight"].t() + sd["bias"]


def pretrain_forward(sd_lf: Dict[str, Tensor], sd_head: Dict[str, Tensor], cfg, a: Dict[str, Tensor],
                     b: Dict[str, Tensor], mlm_a=None, mlm_labels_a=None, mlm_b=None, mlm_labels_b=None):
    """RecformerForPretraining.forward models.py:380-520 at world size 1: contrastive
    CE(cos(z_a, z_b)/temp, arange) + mlm_weight * CE(lm_head(h_mlm), labels, ignore -100) per view.
    Returns (loss, cos_sim, correct_num)."""
    _, z1 = model_forward(sd_lf, cfg, **a)
    _, z2 = model_forward(sd_lf, cfg, **b)
    cos_sim = F.cosine_similarity(z1.unsqueeze(1), z2.unsqueeze(0), dim=-1) / cfg.temp
    labels = torch.arange(cos_sim.size(0))
    loss = F.cross_entropy(cos_sim, labels)
    correct = (cos_sim.argmax(1) == labels).sum()
    for view, ids, lab in ((a, mlm_a, mlm_labels_a), (b, mlm_b, mlm_labels_b)):
        if ids is None or lab is None:
            continue
        h, _ = model_forward(sd_lf, cfg, **dict(view, input_ids=ids))
        scores = lm_head_forward(sd_head, h, cfg.layer_norm_eps)
        loss = loss + cfg.mlm_weight * F.cross_entropy(scores.reshape(-1, scores.shape[-1]), lab.reshape(-1))
    return loss, cos_sim, correct


def ranker_metrics(scores: Tensor, labels: Tensor, ks, max_val: float = 1e4):
    """utils.py:76-108 (Ranker.forward): [ndcg@k, hr@k]... + [MRR, AUC, CE loss]."""
    labels = labels.squeeze()
    loss = F.cross_entropy(scores, labels).item()
    predicts = scores[torch.arange(scores.size(0)), labels].unsqueeze(-1)
    valid_length = (scores > -max_val).sum(-1).float()
    rank = (predicts < scores).sum(-1).float()
    res = []
    for k in ks:
        indicator = (rank < k).float()
        res.append(((1 / torch.log2(rank + 2)) * indicator).mean().item())
        res.append(indicator.mean().item())
    res.append((1 / (rank + 1)).mean().item())
    res.append((1 - (rank / valid_length)).mean().item())
    return res + [loss]
