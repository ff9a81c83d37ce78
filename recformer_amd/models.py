"""Drop-in Recformer model classes on the MI355X HIP kernels.

Mirrors the reference Python API (recformer/models.py): same class names, constructor
arguments, forward() keyword signatures and return types, and the same state-dict keys
(models.py:82-356 plus the transformers Longformer layer names TF:446-1172), so
finetune.py / evaluate_seq.py / checkpoints load unchanged. The arithmetic runs in
hand-written HIP kernels through ops.py; there is no PyTorch/CPU fallback.

Compute dtype: the autocast dtype under a CUDA autocast context (fp16 — torch.cuda.amp's
default, the reference drivers' mode — or bf16), else the parameters' 16-bit type, else fp32
(exact-fp32 MFMA GEMMs); see _compute_dtype.
"""
from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .config import RecformerConfig

__all__ = [
    "RecformerConfig", "RecformerModel", "RecformerForSeqRec", "RecformerForPretraining",
    "RecformerPretrainingOutput", "RecformerModelOutput", "RecformerEmbeddings",
    "RecformerPooler", "Similarity", "create_position_ids_from_input_ids",
]


# ----------------------------------------------------------------------------------
# outputs
class _Output:
    """Tuple/attribute hybrid like transformers' ModelOutput."""

    _fields: Tuple[str, ...] = ()

    def to_tuple(self):
        return tuple(getattr(self, f) for f in self._fields if getattr(self, f) is not None)

    def __getitem__(self, i):
        if isinstance(i, str):
            return getattr(self, i)
        return self.to_tuple()[i]

    def __iter__(self):
        return iter(self.to_tuple())

    def keys(self):
        return [f for f in self._fields if getattr(self, f) is not None]


@dataclass
class RecformerModelOutput(_Output):
    """Fields of LongformerBaseModelOutputWithPooling (TF:79)."""

    last_hidden_state: Optional[torch.Tensor] = None
    pooler_output: Optional[torch.Tensor] = None
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None
    attentions: Optional[Tuple[torch.Tensor, ...]] = None
    global_attentions: Optional[Tuple[torch.Tensor, ...]] = None
    _fields = ("last_hidden_state", "pooler_output", "hidden_states", "attentions", "global_attentions")


LongformerBaseModelOutputWithPooling = RecformerModelOutput


@dataclass
class RecformerPretrainingOutput:
    """models.py:57-66."""

    cl_correct_num: float = 0.0
    cl_total_num: float = 1e-5
    loss: Optional[torch.FloatTensor] = None
    logits: torch.FloatTensor = None
    hidden_states: Optional[Tuple[torch.FloatTensor]] = None
    attentions: Optional[Tuple[torch.FloatTensor]] = None
    global_attentions: Optional[Tuple[torch.FloatTensor]] = None


def create_position_ids_from_input_ids(input_ids, padding_idx):
    """models.py:68-79 (host-side helper kept for API compatibility; the HIP path computes
    the same ids inside rf_prepare_inputs)."""
    mask = input_ids.ne(padding_idx).int()
    incremental_indices = torch.cumsum(mask, dim=1).type_as(mask) * mask
    return incremental_indices.long() + padding_idx


# ----------------------------------------------------------------------------------
# modules (parameter containers with the reference names)
class RecformerEmbeddings(nn.Module):
    """models.py:82-138 — parameter layout only; compute is rf_embed_ln_fwd."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size, padding_idx=config.pad_token_id)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size,
                                                padding_idx=config.pad_token_id)
        self.token_type_embeddings = nn.Embedding(config.token_type_size, config.hidden_size)
        self.item_position_embeddings = nn.Embedding(config.max_item_embeddings, config.hidden_size)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.register_buffer("position_ids", torch.arange(config.max_position_embeddings).expand((1, -1)))
        self.position_embedding_type = getattr(config, "position_embedding_type", "absolute")
        self.padding_idx = config.pad_token_id


class _SelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        d = config.hidden_size
        self.query = nn.Linear(d, d)
        self.key = nn.Linear(d, d)
        self.value = nn.Linear(d, d)
        self.query_global = nn.Linear(d, d)
        self.key_global = nn.Linear(d, d)
        self.value_global = nn.Linear(d, d)


class _DenseLN(nn.Module):
    def __init__(self, d_in, d_out, eps):
        super().__init__()
        self.dense = nn.Linear(d_in, d_out)
        self.LayerNorm = nn.LayerNorm(d_out, eps=eps)


class _Attention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.self = _SelfAttention(config)
        self.output = _DenseLN(config.hidden_size, config.hidden_size, config.layer_norm_eps)


class _Intermediate(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.intermediate_size)


class RecformerLayer(nn.Module):
    """One LongformerLayer (TF:1134-1172) — names match the reference state dict."""

    def __init__(self, config):
        super().__init__()
        self.attention = _Attention(config)
        self.intermediate = _Intermediate(config)
        self.output = _DenseLN(config.intermediate_size, config.hidden_size, config.layer_norm_eps)


class RecformerEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.layer = nn.ModuleList([RecformerLayer(config) for _ in range(config.num_hidden_layers)])


class RecformerPooler(nn.Module):
    """models.py:155-171."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.pooler_type = config.pooler_type

    def forward(self, attention_mask: torch.Tensor, hidden_states: torch.Tensor) -> torch.Tensor:
        if self.pooler_type == "cls":
            return hidden_states[:, 0]
        if self.pooler_type == "avg":
            return (hidden_states * attention_mask.unsqueeze(-1)).sum(1) / attention_mask.sum(-1).unsqueeze(-1)
        raise NotImplementedError


class Similarity(nn.Module):
    """models.py:358-369 — cos(x, y)/temp. Used on the HIP path through ops.cos_scores."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.temp = config.temp

    def forward(self, x, y):
        return nn.functional.cosine_similarity(x, y, dim=-1) / self.temp


def _init_weights(module: nn.Module, std: float) -> None:
    """LongformerPreTrainedModel._init_weights semantics (normal(0, std), zero bias, LN 1/0)."""
    for m in module.modules():
        if isinstance(m, nn.Linear):
            m.weight.data.normal_(0.0, std)
            if m.bias is not None:
                m.bias.data.zero_()
        elif isinstance(m, nn.Embedding):
            m.weight.data.normal_(0.0, std)
            if m.padding_idx is not None:
                m.weight.data[m.padding_idx].zero_()
        elif isinstance(m, nn.LayerNorm):
            m.bias.data.zero_()
            m.weight.data.fill_(1.0)


# ----------------------------------------------------------------------------------
def _needs_grad(module: nn.Module) -> bool:
    """Autograd path when gradients are enabled and some parameter requires them."""
    return torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters())


def _train_path(model: "RecformerModel") -> bool:
    """The training encoder (train.encode_train) when gradients are needed, or when the model is in
    train mode with a nonzero dropout: nn.Dropout applies in train mode whatever the grad mode (the
    reference's model.train() under torch.no_grad() still drops), so the no-grad inference path,
    which has no dropout, is taken only in eval mode or with zero dropout probabilities."""
    if _needs_grad(model):
        return True
    cfg = model.config
    return model.training and (cfg.hidden_dropout_prob > 0 or cfg.attention_probs_dropout_prob > 0)


def _cos_train(z: torch.Tensor, items: torch.Tensor, temp: float) -> torch.Tensor:
    """Differentiable Similarity (models.py:358-369): cos(z_b, items_n) / temp in fp32 (autocast
    computes cosine_similarity in fp32), as normalise + matmul instead of the (B,N,d) broadcast."""
    zn = z.float() / z.float().norm(dim=-1, keepdim=True).clamp_min(1e-8)
    it = items.float()
    itn = it / it.norm(dim=-1, keepdim=True).clamp_min(1e-8)
    with torch.autocast("cuda", enabled=False):
        return (zn @ itn.t()) / temp


# training scoring head (cosine scores + CrossEntropy, models.py:583-599) on the HIP kernels when
# the item table is frozen; False: the torch ops (_cos_train, einsum, F.cross_entropy)
SCORE_HEAD_HIP = True
# bf16 path: keep the fp32 residual stream as split (hi, lo) 16-bit planes;
# False = a plain fp32 tensor plus a separate bf16 GEMM operand (A/B tools, tests).
SPLIT_STREAM = True
# sequences shorter than the 64-token window (catalog items: <s> + <= 63 tokens, finetune.py:38-63)
# not padded at all instead of padded to 64 (rf_band_attn_fwd's short-sequence kernel takes any length
# below the window): the valid rows' outputs are the same (padding is masked), and every GEMM /
# LayerNorm runs on the real rows only (33-token items: 33 rows instead of 64, or 48 at the
# multiple-of-16 padding of round 3)
SHORT_SEQ = True
# run the global fold's pass over h before the qkv GEMM (rf_global_attn_fold_h_stage)
FOLD_EARLY = True
# with FOLD_EARLY: queue the fold's first stage on a side stream that starts once the qkv GEMM is
# done, so its launch-bound projection and its pass over h run beside the HBM-bound band attention
# (the band kernel leaves LDS free on every CU); the main stream joins before the fold's last stage.
# Off: measured slower at C2 (same-process A/B, tools/ab_step.py FOLD_OVERLAP: 13.44 vs 13.20 ms per
# step) — the partial kernel's ~100 KiB-LDS blocks displace band-attention blocks instead of filling
# idle CUs, and the fold's pass over h no longer hits the cache the LayerNorm left it in
FOLD_OVERLAP = False
_SIDE_STREAMS = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(dev)
    return s
# inference callers that read only the pooled CLS vectors (RecformerForSeqRec scores, the catalog
# encoder): the last layer on the CLS rows only when every CLS is a global token (_cls_last_layer)
PRUNE_LAST_LAYER = True
# training: RecformerForPretraining's four encoder passes share one autograd cast per weight
SHARE_TRAIN_CASTS = True
# set by graphs.GraphedForward during capture: the global-slot count of the captured shape, and whether
# every sequence's CLS is global (the CLS-only last layer's condition, read on the host otherwise)
_STATIC_GMAX = None
_STATIC_CLS = None
# read the global-token count after the embedding is queued (False: before the prologue)
ASYNC_GLOBAL_COUNT = True


def _async_count(t: torch.Tensor):
    """Start copying a device integer scalar (or small vector) to pinned host memory (no host wait yet)."""
    buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    buf.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return buf, ev


def _read_count(p):
    buf, ev = p
    ev.synchronize()
    return int(buf) if buf.dim() == 0 else buf.tolist()
# 16-bit inference: the FFN output Linear (K = 3072 -> 768, bias only, TF:1122-1130) as a plain
# library GEMM (torch.addmm -> hipBLASLt, bf16 bias in its epilogue: autocast's Linear does the
# same) instead of rf_gemm; the one layer GEMM without a fused epilogue worth keeping, and the one
# shape where the library's main loop was faster on the same box (profiles/r06/gemm_c2_bar_r06a.jsonl)
FFN2_LIBRARY = False


def _ffn2_library(f: torch.Tensor, lw: dict, tag: str) -> torch.Tensor:
    b = lw.get("b_2_lp")
    if b is None:
        b = lw["b_2_lp"] = lw["b_2"].to(f.dtype)
    with ops._region(tag):
        return torch.addmm(b, f, lw["w_2"].t())


# pretraining training: the LM-head decoder + masked-LM cross entropy on the HIP kernels
# (train._DecoderCE) for 16-bit compute; False = torch ops (F.linear + F.cross_entropy)
DECODER_CE_HIP = True
# pretraining training: the LM head's dense + GELU + LayerNorm on the HIP kernels (16-bit compute,
# train._LMHeadTransform); False = torch ops
LM_HEAD_HIP = True
# pretraining: the LM head runs on the masked (labelled) rows only (_mlm_rows)
LM_HEAD_MASKED_ONLY = True


def _compute_dtype(param_dtype: torch.dtype) -> torch.dtype:
    """The GEMM / attention operand type: the autocast dtype under torch.autocast (fp16 is the
    default of torch.cuda.amp.autocast(), the reference's finetune.py:106-110; bf16 on request),
    else the parameters' type (model.half() / model.to(bfloat16)), else fp32."""
    if torch.is_autocast_enabled("cuda"):
        adt = torch.get_autocast_dtype("cuda")
        return adt if adt in (torch.bfloat16, torch.float16) else torch.bfloat16
    if param_dtype in (torch.bfloat16, torch.float16):
        return param_dtype
    return torch.float32


def _embeds_as_table(inputs_embeds: torch.Tensor, position_ids, pad: int):
    """`inputs_embeds` (B, L, d) as the word table of the embedding kernels: rows pad+1 .. pad+B*L
    hold the vectors in token order and token t's id points at its own row, so rf_embed_ln adds the
    position / type / item-position rows and normalises exactly as for token ids (models.py:106-136,
    `inputs_embeds + position_embeddings + ...`). Rows 0..pad are zero: the padding id the prologue
    writes into the window padding gathers a zero row (those rows are masked keys and are sliced
    off). Gradients reach inputs_embeds through the table. Position ids default to pad+1 .. pad+L
    (create_position_ids_from_inputs_embeds, models.py:140-153)."""
    if inputs_embeds.dim() != 3:
        raise ValueError(f"inputs_embeds must be (batch, seq, hidden), got {tuple(inputs_embeds.shape)}")
    B, L, D = inputs_embeds.shape
    dev = inputs_embeds.device
    table = torch.cat([inputs_embeds.new_zeros(pad + 1, D, dtype=torch.float32),
                       inputs_embeds.reshape(B * L, D).float()], 0)
    ids = torch.arange(pad + 1, pad + 1 + B * L, dtype=torch.int64, device=dev).view(B, L)
    if position_ids is None:
        position_ids = torch.arange(pad + 1, pad + 1 + L, dtype=torch.int64, device=dev).unsqueeze(0).expand(B, L)
    return ids, table, position_ids


def _head_mask_columns(head_mask: Optional[torch.Tensor], cfg) -> Optional[torch.Tensor]:
    """head_mask (num_layers, heads) as per-layer column scales (num_layers, hidden) of the attention
    context: transformers 4.28's LongformerEncoder takes head_mask[layer] and LongformerSelfAttention
    multiplies the local and the global attention probabilities by it per head (the reference passes
    head_mask straight to the encoder, models.py:335-343), which scales that head's context columns."""
    if head_mask is None:
        return None
    nl, H = cfg.num_hidden_layers, cfg.num_attention_heads
    if head_mask.dim() != 2 or tuple(head_mask.shape) != (nl, H):
        raise ValueError(f"head_mask must be (num_hidden_layers, num_attention_heads) = {(nl, H)}, "
                         f"got {tuple(head_mask.shape)}")
    return head_mask.float().repeat_interleave(cfg.hidden_size // H, dim=1)


class _PackedWeights:
    """Compute-dtype copies of the layer weights in the layouts the kernels read.

    Per layer: W_qkv5 = [Wq; Wk; Wv; Wkg; Wvg] (5d x d) so one MFMA GEMM produces q, k, v
    and the global-path k/v over all tokens (TF:504-506, 983-984); biases fp32. Rebuilt
    whenever any parameter's version counter or storage changes (e.g. after an optimizer
    step or load_state_dict).
    """

    def __init__(self):
        self.key = None
        self.data = None

    @staticmethod
    def _sig(model: "RecformerModel", dtype):
        return (dtype,) + tuple((p.data_ptr(), p._version) for p in model.parameters())

    def get(self, model: "RecformerModel", dtype: torch.dtype):
        sig = self._sig(model, dtype)
        if sig != self.key:
            self.data = self._build(model, dtype)
            self.key = sig
        return self.data

    @staticmethod
    @torch.no_grad()
    def _build(model: "RecformerModel", dt: torch.dtype):
        f32 = torch.float32
        emb = model.embeddings
        # embedding tables stay fp32: the reference sums fp32 embeddings even under autocast
        pk = {
            "word": emb.word_embeddings.weight.to(f32).contiguous(),
            "pos": emb.position_embeddings.weight.to(f32).contiguous(),
            "type": emb.token_type_embeddings.weight.to(f32).contiguous(),
            "ipos": emb.item_position_embeddings.weight.to(f32).contiguous(),
            "ln_w": emb.LayerNorm.weight.to(f32).contiguous(),
            "ln_b": emb.LayerNorm.bias.to(f32).contiguous(),
            "layers": [],
        }
        for lyr in model.encoder.layer:
            sa = lyr.attention.self
            lin = [sa.query, sa.key, sa.value, sa.key_global, sa.value_global]
            pk["layers"].append({
                "w_qkv": torch.cat([m.weight for m in lin], 0).to(dt).contiguous(),
                "b_qkv": torch.cat([m.bias for m in lin], 0).to(f32).contiguous(),
                "w_qg": sa.query_global.weight.to(dt).contiguous(),
                "b_qg": sa.query_global.bias.to(f32).contiguous(),
                "w_o": lyr.attention.output.dense.weight.to(dt).contiguous(),
                "b_o": lyr.attention.output.dense.bias.to(f32).contiguous(),
                "ln1_w": lyr.attention.output.LayerNorm.weight.to(f32).contiguous(),
                "ln1_b": lyr.attention.output.LayerNorm.bias.to(f32).contiguous(),
                "w_1": lyr.intermediate.dense.weight.to(dt).contiguous(),
                "b_1": lyr.intermediate.dense.bias.to(f32).contiguous(),
                "w_2": lyr.output.dense.weight.to(dt).contiguous(),
                "b_2": lyr.output.dense.bias.to(f32).contiguous(),
                "ln2_w": lyr.output.LayerNorm.weight.to(f32).contiguous(),
                "ln2_b": lyr.output.LayerNorm.bias.to(f32).contiguous(),
            })
        return pk


class RecformerModel(nn.Module):
    """models.py:174-356 on HIP kernels."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.config = config
        if isinstance(config.attention_window, int):
            assert config.attention_window % 2 == 0, "`config.attention_window` has to be an even value"
            assert config.attention_window > 0, "`config.attention_window` has to be positive"
            config.attention_window = [config.attention_window] * config.num_hidden_layers
        else:
            assert len(config.attention_window) == config.num_hidden_layers, (
                "`len(config.attention_window)` should equal `config.num_hidden_layers`. "
                f"Expected {config.num_hidden_layers}, given {len(config.attention_window)}")
        self.embeddings = RecformerEmbeddings(config)
        self.encoder = RecformerEncoder(config)
        self.pooler = RecformerPooler(config)
        _init_weights(self, config.initializer_range)
        self._packed = _PackedWeights()

    def get_input_embeddings(self):
        return self.embeddings.word_embeddings

    def set_input_embeddings(self, value):
        self.embeddings.word_embeddings = value

    @property
    def dtype(self) -> torch.dtype:
        return self.embeddings.word_embeddings.weight.dtype

    def _window(self) -> int:
        w = self.config.attention_window
        return w if isinstance(w, int) else max(w)

    def forward(
        self,
        input_ids: Optional[torch.Tensor] = None,
        attention_mask: Optional[torch.Tensor] = None,
        global_attention_mask: Optional[torch.Tensor] = None,
        head_mask: Optional[torch.Tensor] = None,
        token_type_ids: Optional[torch.Tensor] = None,
        position_ids: Optional[torch.Tensor] = None,
        item_position_ids: Optional[torch.Tensor] = None,
        inputs_embeds: Optional[torch.Tensor] = None,
        output_attentions: Optional[bool] = None,
        output_hidden_states: Optional[bool] = None,
        return_dict: Optional[bool] = None,
        _pooled_only: bool = False,
    ):
        """models.py:274-356. `_pooled_only` (internal: RecformerForSeqRec and the catalog encoder, which
        read pooler_output only) lets the inference path run the last layer on the CLS rows alone
        (_cls_last_layer); last_hidden_state is then None."""
        cfg = self.config
        output_attentions = output_attentions if output_attentions is not None else cfg.output_attentions
        output_hidden_states = (output_hidden_states if output_hidden_states is not None
                                else cfg.output_hidden_states)
        return_dict = return_dict if return_dict is not None else cfg.use_return_dict
        if input_ids is not None and inputs_embeds is not None:
            raise ValueError("You cannot specify both input_ids and inputs_embeds at the same time")
        if input_ids is None and inputs_embeds is None:
            raise ValueError("You have to specify either input_ids or inputs_embeds")
        word = None
        if inputs_embeds is not None:
            input_ids, word, position_ids = _embeds_as_table(inputs_embeds, position_ids, cfg.pad_token_id)
        head_cols = _head_mask_columns(head_mask, cfg)
        # output_attentions: each layer appends (attentions, global_attentions) recomputed from its
        # input (recformer_amd/probs.py); the kernels themselves never write probabilities
        probe = [] if output_attentions else None
        if _train_path(self):
            # autograd path (recformer_amd/train.py): same kernels, explicit backward
            from .train import encode_train
            last, hidden_all = encode_train(self, input_ids, attention_mask, global_attention_mask,
                                            token_type_ids, position_ids, item_position_ids,
                                            output_hidden_states, word=word, head_cols=head_cols,
                                            attn_probe=probe, pooled_only=_pooled_only)
            if self._last_pruned:
                return RecformerModelOutput(last_hidden_state=None, pooler_output=last)
        else:
            last, hidden_all = self._encode(input_ids, attention_mask, global_attention_mask,
                                            token_type_ids, position_ids, item_position_ids,
                                            output_hidden_states, word=word, head_cols=head_cols,
                                            attn_probe=probe, pooled_only=_pooled_only)
            if self._last_pruned:
                return RecformerModelOutput(last_hidden_state=None, pooler_output=last)
        attentions = global_attentions = None
        if probe is not None:
            attentions = tuple(a for a, _ in probe)
            if any(g is not None for _, g in probe):
                global_attentions = tuple(g for _, g in probe)
        pooled = self.pooler(attention_mask, last)
        if not return_dict:
            out = (last, pooled)
            if output_hidden_states:
                out = out + (hidden_all,)
            if attentions is not None:
                out = out + (attentions,)
            if global_attentions is not None:
                out = out + (global_attentions,)
            return out
        return RecformerModelOutput(last_hidden_state=last, pooler_output=pooled, hidden_states=hidden_all,
                                    attentions=attentions, global_attentions=global_attentions)

    @torch.no_grad()
    def _encode(self, input_ids, attention_mask, global_attention_mask, token_type_ids,
                position_ids, item_position_ids, output_hidden_states, word=None, head_cols=None,
                attn_probe=None, pooled_only=False):
        """(last_hidden_state, hidden_states); with `pooled_only` (callers that read the CLS rows only:
        RecformerForSeqRec, the catalog encoder) it may return (pooled (B, d) fp32, None) instead —
        see the last-layer note below; it says which through self._last_pruned."""
        cfg = self.config
        self._last_pruned = False
        B, L = input_ids.shape
        W = self._window()
        Lp = L + (W - L % W) % W
        windows_all = cfg.window_per_layer()
        if SHORT_SEQ and L < W and W == 64 and all(w == 64 for w in windows_all):
            Lp = L  # no padding rows at all (k_attn_short takes any length below the window)
        D, H = cfg.hidden_size, cfg.num_attention_heads
        hd = D // H
        dt = _compute_dtype(self.dtype)
        pk = self._packed.get(self, dt)

        # number of global slots: one host read per forward (the reference does ~265) — fixed by
        # graphs.GraphedForward while it captures (no host read inside a HIP graph). The count is
        # reduced on the device and copied to pinned memory asynchronously; the host waits for it
        # only after the token streams are prepared and the embedding + LayerNorm is queued, so the
        # GPU has work while the host reads (the global index table is prepared afterwards).
        pending = None
        # pooled_only: whether every sequence's CLS (position 0) is a global token, read with the count
        want_cls = (pooled_only and cfg.pooler_type == "cls" and PRUNE_LAST_LAYER and not output_hidden_states
                    and attn_probe is None)
        cls_global = False
        gstat = None
        if _STATIC_GMAX is not None:
            gmax = _STATIC_GMAX
            cls_global = want_cls and bool(_STATIC_CLS)
        elif global_attention_mask is not None and B > 0:
            if ASYNC_GLOBAL_COUNT:
                # the prologue itself writes each sequence's global count and CLS flag (no mask
                # reductions as separate launches); copied to pinned memory below, read after the
                # embedding is queued
                gstat = torch.empty(B, 2, dtype=torch.int32, device=input_ids.device)
                gmax = 0
            else:
                gm = global_attention_mask != 0
                if attention_mask is not None:
                    gm = gm & (attention_mask > 0)
                gmax = int(gm.sum(1).max().item())
                cls_global = want_cls and bool(gm[:, 0].all())
        else:
            gmax = 0
        ids, pos, tt, ip, flags, gidx = ops.prepare_inputs(
            input_ids, attention_mask, global_attention_mask, token_type_ids, item_position_ids,
            position_ids, Lp, cfg.pad_token_id, gmax, gstat=gstat)
        if gstat is not None:
            pending = _async_count(gstat)

        def _globals():
            # the global index table once the count is known (re-runs the prologue with gmax slots;
            # the token streams it rewrites are identical)
            nonlocal gmax, flags, gidx, cls_global
            if pending is not None:
                st = _read_count(pending)
                gmax = max(c for c, _ in st)
                cls_global = want_cls and all(f for _, f in st)
                if gmax > 0:
                    _, _, _, _, flags, gidx = ops.prepare_inputs(
                        input_ids, attention_mask, global_attention_mask, token_type_ids, item_position_ids,
                        position_ids, Lp, cfg.pad_token_id, gmax)
        # bf16 path: GEMM operands in bf16, residual stream / LN outputs in fp32 (as the
        # reference's autocast run), the fp32 stream held split as (hi, lo) 16-bit planes whose
        # hi plane is the bf16 GEMM operand (ops.add_layernorm_split); fp32 path: everything fp32.
        mixed = dt != torch.float32
        # the split planes' hi half is a bf16 operand; fp16 keeps the fp32 stream plus an fp16 copy
        split = mixed and SPLIT_STREAM and dt == torch.bfloat16
        nl = len(pk["layers"])
        word = pk["word"] if word is None else word
        if split:
            h, h_lo = ops.embed_ln_split(ids, pos, tt, ip, word, pk["pos"], pk["type"], pk["ipos"],
                                         pk["ln_w"], pk["ln_b"], cfg.layer_norm_eps)
            h32 = ops.join_split(h, h_lo) if (output_hidden_states or nl == 0) else None
        else:
            h, h32 = ops.embed_ln(ids, pos, tt, ip, word, pk["pos"], pk["type"], pk["ipos"],
                                  pk["ln_w"], pk["ln_b"], cfg.layer_norm_eps, out_dtype=dt, want_f32=mixed)
            if not mixed:
                h32 = h
        _globals()
        hidden_all = [h32] if output_hidden_states else None
        scale = 1.0 / math.sqrt(hd)
        windows = cfg.window_per_layer()
        # global rows: the key/value-projection fold by default; `config.global_attention_fold
        # = False` keeps the reference's structure (k_g/v_g projected over all tokens).
        fold = getattr(cfg, "global_attention_fold", True)
        eps = cfg.layer_norm_eps
        gws = None
        Lref = L + (W - L % W) % W
        for li, lw in enumerate(pk["layers"]):
            half_w = windows[li] // 2
            if attn_probe is not None:
                from .probs import layer_attention_probs
                attn_probe.append(layer_attention_probs(
                    h, self.encoder.layer[li].attention.self, flags, gidx, B, Lp, L, Lref, H, half_w, scale,
                    None if head_cols is None else head_cols[li, ::hd]))
            nq = 5 * D if (gmax > 0 and not fold) else 3 * D
            gargs = (h, lw["w_qg"], lw["b_qg"], scale, lw["w_qkv"][3 * D:4 * D], lw["b_qkv"][3 * D:4 * D],
                     lw["w_qkv"][4 * D:5 * D], lw["b_qkv"][4 * D:5 * D], flags, gidx, B, Lp, H)
            early = gmax > 0 and fold and FOLD_EARLY
            if li == nl - 1 and cls_global and gmax > 0 and fold and h.is_cuda:
                self._last_pruned = True
                return _cls_last_layer(self, lw, gargs, gws, h, h_lo if split else None, h32, head_cols, li,
                                       B, Lp, D, H, dt, mixed), None
            side = early and FOLD_OVERLAP and h.is_cuda
            if early:
                if gws is None:
                    gws = ops.global_fold_workspace(h, B, Lp, H, gmax)
                if not side:
                    # the fold's pass over h while h is still cache-resident from the LayerNorm
                    # that wrote it; its last stage runs after the local attention has written ctx
                    ops.global_attention_fold_h_stage(1, gws, *gargs, tag="global_attn")
            qkv = ops.gemm(h, lw["w_qkv"][:nq], lw["b_qkv"][:nq], ops.RF_EPI_BIAS,
                           scale_cols=D, col_scale=scale, tag="gemm_qkv")
            if side:
                # stage 1 beside the band attention; h and gws stay alive and unwritten until the
                # main stream has joined (the next writer of h is this layer's LayerNorm)
                main_s = torch.cuda.current_stream(h.device)
                side_s = _side_stream(h.device)
                side_s.wait_stream(main_s)
                with torch.cuda.stream(side_s):
                    ops.global_attention_fold_h_stage(1, gws, *gargs, tag="global_attn")
            ctx = ops.band_attention(qkv[:, 0:D], qkv[:, D:2 * D], qkv[:, 2 * D:3 * D], flags,
                                     gidx, B, Lp, H, half_w, tag="band_attn")
            if side:
                main_s.wait_stream(side_s)
            if early:
                ops.global_attention_fold_h_stage(2, gws, *gargs, out=ctx, tag="global_attn")
            elif gmax > 0:
                if fold:
                    ops.global_attention_fold_h(h, lw["w_qg"], lw["b_qg"], scale, lw["w_qkv"][3 * D:4 * D],
                                                lw["b_qkv"][3 * D:4 * D], lw["w_qkv"][4 * D:5 * D],
                                                lw["b_qkv"][4 * D:5 * D], flags, gidx, B, Lp, H, ctx,
                                                tag="global_attn")
                else:
                    hg = ops.gather_global_rows(h, gidx, B, Lp)
                    qg = ops.gemm(hg, lw["w_qg"], lw["b_qg"], ops.RF_EPI_BIAS, scale_cols=D, col_scale=scale)
                    ops.global_attention(qg, qkv[:, 3 * D:4 * D], qkv[:, 4 * D:5 * D], flags, gidx,
                                         B, Lp, H, ctx, tag="global_attn")
            w_o = lw["w_o"]
            if head_cols is not None:
                # head_mask (TF 4.28 LongformerSelfAttention: probs * layer_head_mask, local and global)
                # scales each head's context columns: folded into the output projection's input columns
                w_o = (w_o.float() * head_cols[li]).to(w_o.dtype).contiguous()
            if not mixed:
                t = ops.gemm(ctx, w_o, lw["b_o"], ops.RF_EPI_BIAS_RESID, resid=h32,
                             tag="gemm_out")
                a = ops.layernorm(t, lw["ln1_w"], lw["ln1_b"], eps, out=t, tag="layernorm")
                f = ops.gemm(a, lw["w_1"], lw["b_1"], ops.RF_EPI_BIAS_GELU, tag="gemm_ffn1")
                t2 = ops.gemm(f, lw["w_2"], lw["b_2"], ops.RF_EPI_BIAS_RESID, resid=a, tag="gemm_ffn2")
                h = h32 = ops.layernorm(t2, lw["ln2_w"], lw["ln2_b"], eps, out=t2, tag="layernorm")
            elif split:
                # bf16 path, the reference under autocast: each dense output is bf16 (the GEMM
                # epilogue rounds it, as autocast's Linear does), the residual stream and the
                # LayerNorm are fp32 (TF:1064-1071, 1123-1130): LN(bf16 dense + fp32 stream),
                # the stream updated in place as planes (h = its hi plane); the last layer (and
                # every layer when hidden states are returned) also writes the fp32 output.
                last_layer = li == nl - 1
                t = ops.gemm(ctx, w_o, lw["b_o"], ops.RF_EPI_BIAS, tag="gemm_out")
                ops.add_layernorm_split(t, h, h_lo, lw["ln1_w"], lw["ln1_b"], eps, tag="layernorm")
                f = ops.gemm(h, lw["w_1"], lw["b_1"], ops.RF_EPI_BIAS_GELU, tag="gemm_ffn1")
                if FFN2_LIBRARY:
                    t2 = _ffn2_library(f, lw, "gemm_ffn2")
                else:
                    t2 = ops.gemm(f, lw["w_2"], lw["b_2"], ops.RF_EPI_BIAS, tag="gemm_ffn2")
                _, _, h32 = ops.add_layernorm_split(t2, h, h_lo, lw["ln2_w"], lw["ln2_b"], eps,
                                                    planes=not last_layer,
                                                    want_f32=last_layer or output_hidden_states,
                                                    tag="layernorm")
            else:
                # the same with the fp32 stream as a plain fp32 tensor (SPLIT_STREAM = False)
                t = ops.gemm(ctx, w_o, lw["b_o"], ops.RF_EPI_BIAS, tag="gemm_out")
                a, a32 = ops.add_layernorm(t, h32, lw["ln1_w"], lw["ln1_b"], eps, out_dtype=dt,
                                           res_out=None if output_hidden_states else h32, tag="layernorm")
                f = ops.gemm(a, lw["w_1"], lw["b_1"], ops.RF_EPI_BIAS_GELU, tag="gemm_ffn1")
                t2 = ops.gemm(f, lw["w_2"], lw["b_2"], ops.RF_EPI_BIAS, tag="gemm_ffn2")
                h, h32 = ops.add_layernorm(t2, a32, lw["ln2_w"], lw["ln2_b"], eps, out_dtype=dt, res_out=a32,
                                           tag="layernorm")
            if output_hidden_states:
                hidden_all.append(h32)
        last = h32.view(B, Lp, D)[:, :L]
        if output_hidden_states:
            hidden_all = tuple(x.view(B, Lp, D)[:, :L] for x in hidden_all)
        return last, hidden_all


def _cls_last_layer(model, lw, gargs, gws, h, h_lo, h32, head_cols, li, B, Lp, D, H, dt, mixed):
    """The last layer on the CLS rows only (RecformerModel._encode with pooled_only).

    The pooler reads row 0 of the last layer's output (models.py:160-171) and RecformerForSeqRec /
    the catalog encoder read nothing else (similarity_score and the loss, models.py:539-599;
    finetune.py:38-63). Each output row of a layer depends on the other rows only through attention;
    a global token's attention output is the global path's (TF:612-629), which the fold computes from
    the layer input h alone. So with every CLS global the last layer is: the fold, then the output
    projection, residual LayerNorm, FFN and LayerNorm on the B CLS rows — the same arithmetic as the
    full layer for those rows, without the qkv GEMM, the band attention and the other B(Lp-1) rows.
    Returns the pooled vectors (B, d) fp32."""
    eps = model.config.layer_norm_eps
    dev = h.device
    if gws is None:
        gws = ops.global_fold_workspace(h, B, Lp, H, gargs[9].shape[1])  # gargs[9]: gidx
    ctx = torch.empty(B * Lp, D, dtype=h.dtype, device=dev)  # the fold writes the global rows only
    ops.global_attention_fold_h_stage(1, gws, *gargs, tag="global_attn")
    ops.global_attention_fold_h_stage(2, gws, *gargs, out=ctx, tag="global_attn")
    rows = torch.arange(B, device=dev) * Lp
    c = ctx.index_select(0, rows)
    if h_lo is not None:
        res = ops.join_split(h.index_select(0, rows), h_lo.index_select(0, rows))
    else:
        res = h32.index_select(0, rows).float().contiguous()
    w_o = lw["w_o"]
    if head_cols is not None:
        w_o = (w_o.float() * head_cols[li]).to(w_o.dtype).contiguous()
    if not mixed:
        t = ops.gemm(c, w_o, lw["b_o"], ops.RF_EPI_BIAS_RESID, resid=res, tag="cls_gemm_out")
        a = ops.layernorm(t, lw["ln1_w"], lw["ln1_b"], eps, out=t, tag="cls_layernorm")
        f = ops.gemm(a, lw["w_1"], lw["b_1"], ops.RF_EPI_BIAS_GELU, tag="cls_gemm_ffn1")
        t2 = ops.gemm(f, lw["w_2"], lw["b_2"], ops.RF_EPI_BIAS_RESID, resid=a, tag="cls_gemm_ffn2")
        return ops.layernorm(t2, lw["ln2_w"], lw["ln2_b"], eps, out=t2, tag="cls_layernorm")
    t = ops.gemm(c, w_o, lw["b_o"], ops.RF_EPI_BIAS, tag="cls_gemm_out")
    a, a32 = ops.add_layernorm(t, res, lw["ln1_w"], lw["ln1_b"], eps, out_dtype=dt, tag="cls_layernorm")
    f = ops.gemm(a, lw["w_1"], lw["b_1"], ops.RF_EPI_BIAS_GELU, tag="cls_gemm_ffn1")
    t2 = ops.gemm(f, lw["w_2"], lw["b_2"], ops.RF_EPI_BIAS, tag="cls_gemm_ffn2")
    _, y32 = ops.add_layernorm(t2, a32, lw["ln2_w"], lw["ln2_b"], eps, out_dtype=dt, tag="cls_layernorm")
    return y32


def _negatives(cfg, batch_size: int, device) -> torch.Tensor:
    """Sampled-softmax negatives (models.py:594): torch.randint on the CPU global RNG, as the reference,
    then copied to the device; inside a HIP-graph capture (graphs.CapturedTrainStep) on the device's
    generator instead (graph-safe philox offsets: fresh negatives on every replay), since a host tensor
    cannot enter a captured graph."""
    size = (batch_size, cfg.finetune_negative_sample_size)
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        return torch.randint(0, cfg.item_num, size, device=device)
    return torch.randint(0, cfg.item_num, size).to(device)


class RecformerForSeqRec(nn.Module):
    """models.py:524-599 on HIP kernels (scores via normalize + MFMA GEMM, never the
    (B,N,d) broadcast of nn.CosineSimilarity)."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.config = config
        self.longformer = RecformerModel(config)
        self.sim = Similarity(config)
        self._item_cache_key = None
        self._item_cache = None

    def init_item_embedding(self, embeddings: Optional[torch.Tensor] = None):
        """models.py:533-537."""
        self.item_embedding = nn.Embedding(num_embeddings=self.config.item_num,
                                           embedding_dim=self.config.hidden_size)
        if embeddings is not None:
            self.item_embedding = nn.Embedding.from_pretrained(embeddings, freeze=True)
            print("Initalize item embeddings from vectors.")
        self._item_cache_key = None

    def _items(self, dt: torch.dtype):
        w = self.item_embedding.weight
        key = (w.data_ptr(), w._version, dt, w.device)
        if key != self._item_cache_key:
            with torch.no_grad():
                table = w.detach().to(dt).contiguous()
                self._item_cache = (table, ops.row_inv_norm(table))
            self._item_cache_key = key
        return self._item_cache

    def similarity_score(self, pooler_output, candidates=None):
        """models.py:539-545: (B,N) or (B,C) fp32 scores = cos / temp."""
        dt = pooler_output.dtype
        z = pooler_output.to(dt).contiguous()
        table, rnorm = self._items(dt)
        inv_t = 1.0 / self.config.temp
        if candidates is None:
            return ops.cos_scores(z, table, inv_t, items_rnorm=rnorm)
        return ops.cos_scores_cand(z, table, candidates, inv_t, items_rnorm=rnorm)

    def forward(self, input_ids=None, attention_mask=None, global_attention_mask=None, head_mask=None,
                token_type_ids=None, position_ids=None, item_position_ids=None, inputs_embeds=None,
                output_attentions=None, output_hidden_states=None, return_dict=None, candidates=None,
                labels=None):
        batch_size = input_ids.size(0)
        outputs = self.longformer(input_ids, attention_mask=attention_mask,
                                  global_attention_mask=global_attention_mask, head_mask=head_mask,
                                  token_type_ids=token_type_ids, position_ids=position_ids,
                                  item_position_ids=item_position_ids, inputs_embeds=inputs_embeds,
                                  output_attentions=output_attentions,
                                  output_hidden_states=output_hidden_states, return_dict=True,
                                  _pooled_only=True)
        pooler_output = outputs.pooler_output
        if _needs_grad(self) and SCORE_HEAD_HIP and not self.item_embedding.weight.requires_grad and \
                pooler_output.is_cuda:
            # training head on HIP (models.py:583-599): fp32 cosine scores against the frozen table
            # (from_pretrained(freeze=True), models.py:536) with its inverse norms cached once, the
            # backward's dz on rf_cos_score_bwd, the CrossEntropy on rf_cross_entropy_fwd / _bwd
            from . import train
            table, rnorm = self._items(torch.float32)
            inv_t = 1.0 / self.config.temp
            if labels is None:
                return train.cos_scores_train(pooler_output, table, rnorm, inv_t, candidates)
            if self.config.finetune_negative_sample_size <= 0:
                return train.cross_entropy_train(train.cos_scores_train(pooler_output, table, rnorm, inv_t), labels)
            candidates = torch.cat((labels.unsqueeze(-1), _negatives(self.config, batch_size, labels.device)), dim=-1)
            logits = train.cos_scores_train(pooler_output, table, rnorm, inv_t, candidates)
            return train.cross_entropy_train(logits, torch.zeros_like(labels))
        if _needs_grad(self):
            # training head: differentiable cosine scores + CrossEntropy (models.py:583-599) as torch
            # ops — a trainable item table (init_item_embedding() without vectors)
            table = self.item_embedding.weight
            if labels is None:
                items = table if candidates is None else table[candidates]
                return (_cos_train(pooler_output, items, self.config.temp) if candidates is None else
                        torch.einsum("bd,bcd->bc", F.normalize(pooler_output.float(), dim=-1, eps=1e-8),
                                     F.normalize(items.float(), dim=-1, eps=1e-8)) / self.config.temp)
            if self.config.finetune_negative_sample_size <= 0:
                return F.cross_entropy(_cos_train(pooler_output, table, self.config.temp), labels)
            candidates = torch.cat((labels.unsqueeze(-1), _negatives(self.config, batch_size, labels.device)), dim=-1)
            items = table[candidates].float()
            zn = F.normalize(pooler_output.float(), dim=-1, eps=1e-8)
            logits = torch.einsum("bd,bcd->bc", zn, F.normalize(items, dim=-1, eps=1e-8)) / self.config.temp
            return F.cross_entropy(logits, torch.zeros_like(labels))
        if labels is None:
            return self.similarity_score(pooler_output, candidates)
        if self.config.finetune_negative_sample_size <= 0:
            logits = self.similarity_score(pooler_output)
            return ops.cross_entropy(logits, labels)  # CrossEntropyLoss, models.py:589-591
        # sampled softmax: candidates from the CPU global RNG as models.py:594
        candidates = torch.cat((labels.unsqueeze(-1), _negatives(self.config, batch_size, labels.device)), dim=-1)
        logits = self.similarity_score(pooler_output, candidates)
        target = torch.zeros_like(labels, device=labels.device)
        return ops.cross_entropy(logits, target)  # models.py:595-597


class RecformerForPretraining(nn.Module):
    """models.py:370-520: two-view contrastive loss (cos(z_a, z_b) / temp, CrossEntropy against
    arange, cl_correct_num) plus mlm_weight x the masked-LM losses of LongformerLMHead
    (TF:1265-1285: dense -> exact GELU -> LayerNorm -> decoder) on the MLM-input encodings.
    Inference: every encoder pass, the head's GEMMs / LayerNorm and both cross entropies run on
    the HIP kernels. Training (gradients enabled): the encoder runs through recformer_amd/train.py
    and the heads are differentiable torch ops; under torch.distributed the z vectors are
    all-gathered across ranks with the local slot keeping its graph (models.py:474-490)."""

    def __init__(self, config: RecformerConfig):
        super().__init__()
        self.config = config
        self.longformer = RecformerModel(config)
        self.lm_head = _LMHead(config)
        self.sim = Similarity(config)
        self._head_key = None
        self._head = None

    def _head_weights(self, dt: torch.dtype):
        m = self.lm_head
        key = (dt,) + tuple((p.data_ptr(), p._version) for p in m.parameters())
        if key != self._head_key:
            with torch.no_grad():
                self._head = {
                    "w_d": m.dense.weight.to(dt).contiguous(), "b_d": m.dense.bias.float().contiguous(),
                    "ln_w": m.layer_norm.weight.float().contiguous(), "ln_b": m.layer_norm.bias.float().contiguous(),
                    "w_dec": m.decoder.weight.to(dt).contiguous(), "b_dec": m.decoder.bias.float().contiguous(),
                }
            self._head_key = key
        return self._head

    def lm_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """LongformerLMHead.forward (TF:1277-1285) -> (B*L, vocab) logits in the compute dtype."""
        dt = _compute_dtype(self.longformer.dtype)
        w = self._head_weights(dt)
        x = hidden.reshape(-1, hidden.shape[-1]).to(dt).contiguous()
        t = ops.gemm(x, w["w_d"], w["b_d"], ops.RF_EPI_BIAS_GELU)
        t = ops.layernorm(t, w["ln_w"], w["ln_b"], self.config.layer_norm_eps)
        return ops.gemm(t, w["w_dec"], w["b_dec"], ops.RF_EPI_BIAS)

    def forward(self, input_ids_a=None, attention_mask_a=None, global_attention_mask_a=None,
                token_type_ids_a=None, item_position_ids_a=None, mlm_input_ids_a=None, mlm_labels_a=None,
                input_ids_b=None, attention_mask_b=None, global_attention_mask_b=None, token_type_ids_b=None,
                item_position_ids_b=None, mlm_input_ids_b=None, mlm_labels_b=None, head_mask=None,
                position_ids=None, inputs_embeds=None, labels=None, output_attentions=None,
                output_hidden_states=None, return_dict=None):
        batch_size = input_ids_a.size(0)

        def enc(ids, am, gm, tt, ip):
            return self.longformer(ids, attention_mask=am, global_attention_mask=gm, head_mask=head_mask,
                                   token_type_ids=tt, position_ids=position_ids, item_position_ids=ip,
                                   inputs_embeds=inputs_embeds, output_attentions=output_attentions,
                                   output_hidden_states=output_hidden_states, return_dict=True)

        # training: the four passes share one autograd cast per weight (train.shared_casts)
        share = contextlib.nullcontext()
        if _needs_grad(self) and SHARE_TRAIN_CASTS:
            from .train import shared_casts
            share = shared_casts()
        with share:
            outputs_a = enc(input_ids_a, attention_mask_a, global_attention_mask_a, token_type_ids_a,
                            item_position_ids_a)
            outputs_b = enc(input_ids_b, attention_mask_b, global_attention_mask_b, token_type_ids_b,
                            item_position_ids_b)
            mlm_outputs_a = (enc(mlm_input_ids_a, attention_mask_a, global_attention_mask_a, token_type_ids_a,
                                 item_position_ids_a) if mlm_input_ids_a is not None else None)
            mlm_outputs_b = (enc(mlm_input_ids_b, attention_mask_b, global_attention_mask_b, token_type_ids_b,
                                 item_position_ids_b) if mlm_input_ids_b is not None else None)

        z1, z2 = outputs_a.pooler_output, outputs_b.pooler_output
        if _needs_grad(self) or self.training:
            # train mode (with or without gradients, like the reference's modules): the z all-gather
            # across ranks and the differentiable heads
            return self._train_losses(z1, z2, outputs_a, mlm_outputs_a, mlm_labels_a, mlm_outputs_b,
                                      mlm_labels_b, batch_size)
        dt = _compute_dtype(self.longformer.dtype)
        z1c, z2c = z1.to(dt).contiguous(), z2.to(dt).contiguous()
        cos_sim = ops.cos_scores(z1c, z2c, 1.0 / self.config.temp)  # Similarity(z1[:,None], z2[None])
        cl_labels = torch.arange(cos_sim.size(0), device=cos_sim.device)
        loss, amax = ops.cross_entropy(cos_sim, cl_labels, want_argmax=True)
        correct_num = (amax == cl_labels).sum()
        for mo, ml in ((mlm_outputs_a, mlm_labels_a), (mlm_outputs_b, mlm_labels_b)):
            if mo is not None and ml is not None:
                hid, lab = _mlm_rows(mo.last_hidden_state, ml)
                scores = self.lm_logits(hid)
                loss = loss + self.config.mlm_weight * ops.cross_entropy(scores, lab)
        return RecformerPretrainingOutput(loss=loss, logits=cos_sim, cl_correct_num=correct_num,
                                          cl_total_num=batch_size, hidden_states=outputs_a.hidden_states,
                                          attentions=outputs_a.attentions,
                                          global_attentions=outputs_a.global_attentions)


# Row capacity of the masked-LM head in a captured training step (set by recformer_amd.graphs)
_STATIC_MLM_ROWS: Optional[int] = None


def _mlm_rows(hidden: torch.Tensor, labels: torch.Tensor):
    """The rows the masked-LM loss reads: CrossEntropyLoss ignores label -100
    (models.py:499-510), so the LM head over only the labelled rows gives the same loss as over
    every token, at ~15% of the head's GEMM work and logits memory. One host read (the row count)
    per call. LM_HEAD_MASKED_ONLY = False (or no labelled row) keeps every row."""
    h = hidden.reshape(-1, hidden.shape[-1])
    lab = labels.reshape(-1)
    if not LM_HEAD_MASKED_ONLY:
        return h, lab
    if _STATIC_MLM_ROWS is not None:
        # captured step (recformer_amd.graphs): a fixed row count without a host read — the labelled
        # rows first, in order (a stable sort of the ignore flag), then unlabelled rows (label -100,
        # ignored by the CE) up to the capacity
        cap = min(_STATIC_MLM_ROWS, lab.numel())
        sel = torch.argsort((lab == -100).to(torch.uint8), stable=True)[:cap]
        return h.index_select(0, sel), lab.index_select(0, sel)
    sel = (lab != -100).nonzero().squeeze(1)
    if sel.numel() == 0:
        return h, lab
    return h.index_select(0, sel), lab.index_select(0, sel)


def _pretrain_train_losses(self, z1, z2, outputs_a, mlm_a, lab_a, mlm_b, lab_b, batch_size):
    """Differentiable losses of models.py:472-510 (training): all_gather of z across ranks (the
    local slot keeps its graph, models.py:474-490), contrastive CE, LM head + masked-LM CE."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and self.training:
        ws, rk = dist.get_world_size(), dist.get_rank()
        z1_list = [torch.zeros_like(z1) for _ in range(ws)]
        z2_list = [torch.zeros_like(z2) for _ in range(ws)]
        dist.all_gather(z1_list, z1.contiguous())
        dist.all_gather(z2_list, z2.contiguous())
        z1_list[rk] = z1
        z2_list[rk] = z2
        z1 = torch.cat(z1_list, 0)
        z2 = torch.cat(z2_list, 0)
    cos_sim = _cos_train(z1, z2, self.config.temp)
    labels = torch.arange(cos_sim.size(0), device=cos_sim.device)
    loss = F.cross_entropy(cos_sim, labels)
    correct_num = (torch.argmax(cos_sim, 1) == labels).sum()
    head = self.lm_head
    for mo, ml in ((mlm_a, lab_a), (mlm_b, lab_b)):
        if mo is not None and ml is not None:
            hid, lab = _mlm_rows(mo.last_hidden_state, ml)
            dt = _compute_dtype(self.longformer.dtype)
            hip = hid.is_cuda and dt != torch.float32 and hid.shape[-1] % 64 == 0
            if hip and LM_HEAD_HIP:
                # dense + GELU + LayerNorm on the HIP kernels (train._LMHeadTransform)
                from .train import lm_head_transform
                x = lm_head_transform(hid.to(dt), head.dense.weight, head.dense.bias, head.layer_norm.weight,
                                      head.layer_norm.bias, self.config.layer_norm_eps)
            else:
                x = F.gelu(F.linear(hid, head.dense.weight, head.dense.bias))
                x = F.layer_norm(x, (x.shape[-1],), head.layer_norm.weight, head.layer_norm.bias,
                                 self.config.layer_norm_eps)
            if hip and DECODER_CE_HIP:
                # decoder GEMM + CE + its backward on the HIP kernels (train._DecoderCE)
                from .train import decoder_ce
                mlm = decoder_ce(x.to(dt), head.decoder.weight, head.bias, lab)
            else:
                scores = F.linear(x, head.decoder.weight, head.bias)
                mlm = F.cross_entropy(scores.reshape(-1, self.config.vocab_size), lab)
            loss = loss + self.config.mlm_weight * mlm
    return RecformerPretrainingOutput(loss=loss, logits=cos_sim, cl_correct_num=correct_num,
                                      cl_total_num=batch_size, hidden_states=outputs_a.hidden_states,
                                      attentions=outputs_a.attentions, global_attentions=outputs_a.global_attentions)


RecformerForPretraining._train_losses = _pretrain_train_losses


class _LMHead(nn.Module):
    """LongformerLMHead parameter names (TF:1265-1285): dense, layer_norm, decoder, bias."""

    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.decoder = nn.Linear(config.hidden_size, config.vocab_size)
        self.bias = nn.Parameter(torch.zeros(config.vocab_size))
        self.decoder.bias = self.bias
