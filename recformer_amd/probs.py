"""Attention probabilities for `output_attentions=True` (a diagnostic output).

The encoder's band / global attention kernels never write their probabilities: softmax rows live
in registers and only the context reaches HBM. When a caller asks for them, each layer recomputes
them from its input h: the q / k / query_global / key_global projections on the HIP GEMM
(ops.gemm), the banded scores, masking and softmax as torch ops on the device, laid out as
transformers 4.28's LongformerSelfAttention returns them (the version the reference pins;
models.py:335-355 passes them through):

  attentions[l]        (B, H, L, G + 2w + 1): G global-key columns (local keys at the global
                       positions, TF:869-926), then the band columns for key offsets -w..w
                       (_sliding_chunks_query_key_matmul, TF:759-823); keys that are global or
                       padding are masked out of the band; padded and global query rows are zero
                       (TF:574-579, 626-629);
                       cropped to the L input rows (LongformerEncoder, TF:1229-1236).
  global_attentions[l] (B, H, Lp, G), Lp = L padded to the window: softmax(qg . kg) of each global
                       query over the valid keys (TF:964-1013), transposed as the encoder does; an
                       empty global slot's row is uniform over Lp, as the reference's all-min score
                       row softmaxes to.

Both are multiplied by the layer's head_mask row when one is given. They are the probabilities
before attention dropout (the kernels' dropout mask is their own counter hash, not torch's RNG).
Cost: four extra projections and a (H, L, 2w+1) score block per sequence per layer — a debugging
aid, not a hot path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import ops


def _proj(h: torch.Tensor, lin: torch.nn.Linear, dt: torch.dtype, scale: float = 1.0) -> torch.Tensor:
    w = lin.weight.detach().to(dt).contiguous()
    b = lin.bias.detach().float().contiguous()
    D = w.shape[0]
    if scale != 1.0:
        return ops.gemm(h, w, b, ops.RF_EPI_BIAS, scale_cols=D, col_scale=scale)
    return ops.gemm(h, w, b, ops.RF_EPI_BIAS)


@torch.no_grad()
def layer_attention_probs(h: torch.Tensor, self_attn, flags: torch.Tensor, gidx: torch.Tensor, B: int,
                          Lp: int, L: int, Lref: int, H: int, half_w: int, scale: float,
                          head_mask: Optional[torch.Tensor] = None
                          ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """(attentions, global_attentions or None) of one layer from its input h (B*Lp, d) in the
    compute dtype. `self_attn` holds the query/key/query_global/key_global Linears; flags (B, Lp)
    0 padding / 1 local / 2 global; gidx (B, G) global positions, -1 for empty slots."""
    dt = h.dtype
    D = h.shape[1]
    hd = D // H
    w = half_w
    nb = 2 * w + 1
    q = _proj(h, self_attn.query, dt, scale).float().view(B, Lp, H, hd).permute(0, 2, 1, 3)
    k = _proj(h, self_attn.key, dt).float().view(B, Lp, H, hd).permute(0, 2, 1, 3)
    fl = flags.view(B, Lp)
    G = gidx.shape[1]
    hm = head_mask.float().view(H, 1, 1) if head_mask is not None else None
    neg = float("-inf")
    local = []
    for b in range(B):
        kb = F.pad(k[b], (0, 0, w, w)).unfold(1, nb, 1)               # (H, Lp, hd, nb)
        s = torch.matmul(q[b, :, :L].unsqueeze(2), kb[:, :L]).squeeze(2)  # (H, L, nb)
        ok = F.pad(fl[b] == 1, (w, w), value=False).unfold(0, nb, 1)[:L]  # (L, nb)
        s = s.masked_fill(~ok.unsqueeze(0), neg)
        if G > 0:
            gi = gidx[b].long()
            kg = k[b][:, gi.clamp(min=0)]                             # (H, G, hd)
            sg = torch.matmul(q[b, :, :L], kg.transpose(-1, -2))      # (H, L, G)
            sg = sg.masked_fill((gi < 0).view(1, 1, G), neg)
            s = torch.cat([sg, s], dim=-1)
        p = torch.softmax(s, dim=-1).nan_to_num_(0.0)
        # padded query rows, and global query rows (their output is the global path's; TF:626-629)
        p = p.masked_fill((fl[b, :L] != 1).view(1, L, 1), 0.0)
        if hm is not None:
            p = p * hm
        local.append(p)
    attentions = torch.stack(local).to(dt)
    if G == 0:
        return attentions, None
    rows = (torch.arange(B, device=h.device).view(B, 1) * Lp + gidx.long().clamp(min=0)).reshape(-1)
    qg = _proj(h[rows].contiguous(), self_attn.query_global, dt, scale).float().view(B, G, H, hd).transpose(1, 2)
    kg = _proj(h, self_attn.key_global, dt).float().view(B, Lp, H, hd).permute(0, 2, 1, 3)
    sg = torch.matmul(qg, kg.transpose(-1, -2))                       # (B, H, G, Lp)
    sg = sg.masked_fill((fl == 0).view(B, 1, 1, Lp), neg)
    if Lref > Lp:
        sg = F.pad(sg, (0, Lref - Lp), value=neg)
    elif Lref < Lp:
        sg = sg[..., :Lref]
    pg = torch.softmax(sg, dim=-1)
    empty = (gidx < 0).view(B, 1, G, 1)
    pg = torch.where(empty, torch.full_like(pg, 1.0 / Lref), pg)
    if hm is not None:
        pg = pg * hm.view(1, H, 1, 1)
    return attentions, pg.transpose(2, 3).to(dt)
