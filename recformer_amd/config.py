"""RecformerConfig — standalone, attribute- and keyword-compatible with the reference.

Reference: recformer/models.py:24-55 (`RecformerConfig(LongformerConfig)`), whose
Longformer defaults come from transformers' `LongformerConfig`
(configuration_longformer.py). Callers (finetune.py:202-209,
lightning_pretrain.py:58-63) do `RecformerConfig.from_pretrained(
'allenai/longformer-base-4096')` and then overwrite attributes; that name resolves
offline here to the literal longformer-base-4096 hyper-parameters below, so no hub
access is needed.
"""
from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, List, Union

# allenai/longformer-base-4096 config.json, written out literally (SURVEY.md §8c:
# hub fetches are unavailable offline).
LONGFORMER_BASE_4096: Dict[str, Any] = dict(
    vocab_size=50265,
    hidden_size=768,
    num_hidden_layers=12,
    num_attention_heads=12,
    intermediate_size=3072,
    hidden_act="gelu",
    hidden_dropout_prob=0.1,
    attention_probs_dropout_prob=0.1,
    max_position_embeddings=4098,
    type_vocab_size=1,
    initializer_range=0.02,
    layer_norm_eps=1e-5,
    pad_token_id=1,
    bos_token_id=0,
    eos_token_id=2,
    sep_token_id=2,
    attention_window=[512] * 12,
    onnx_export=False,
)

_PRESETS = {
    "allenai/longformer-base-4096": LONGFORMER_BASE_4096,
    "longformer-base-4096": LONGFORMER_BASE_4096,
}


class RecformerConfig:
    """Hyper-parameters read by the hot path."""

    model_type = "recformer"

    def __init__(
        self,
        attention_window: Union[List[int], int] = 64,
        sep_token_id: int = 2,
        token_type_size: int = 4,
        max_token_num: int = 2048,
        max_item_embeddings: int = 32,
        max_attr_num: int = 12,
        max_attr_length: int = 8,
        pooler_type: str = "cls",
        temp: float = 0.05,
        mlm_weight: float = 0.1,
        item_num: int = 0,
        finetune_negative_sample_size: int = 0,
        # Longformer / BERT fields (transformers LongformerConfig defaults)
        vocab_size: int = 30522,
        hidden_size: int = 768,
        num_hidden_layers: int = 12,
        num_attention_heads: int = 12,
        intermediate_size: int = 3072,
        hidden_act: str = "gelu",
        hidden_dropout_prob: float = 0.1,
        attention_probs_dropout_prob: float = 0.1,
        max_position_embeddings: int = 512,
        type_vocab_size: int = 2,
        initializer_range: float = 0.02,
        layer_norm_eps: float = 1e-12,
        pad_token_id: int = 1,
        bos_token_id: int = 0,
        eos_token_id: int = 2,
        onnx_export: bool = False,
        output_attentions: bool = False,
        output_hidden_states: bool = False,
        use_return_dict: bool = True,
        chunk_size_feed_forward: int = 0,
        **kwargs: Any,
    ):
        self.attention_window = attention_window
        self.sep_token_id = sep_token_id
        self.token_type_size = token_type_size
        self.max_token_num = max_token_num
        self.max_item_embeddings = max_item_embeddings
        self.max_attr_num = max_attr_num
        self.max_attr_length = max_attr_length
        self.pooler_type = pooler_type
        self.temp = temp
        self.mlm_weight = mlm_weight
        self.item_num = item_num
        self.finetune_negative_sample_size = finetune_negative_sample_size
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.intermediate_size = intermediate_size
        self.hidden_act = hidden_act
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.initializer_range = initializer_range
        self.layer_norm_eps = layer_norm_eps
        self.pad_token_id = pad_token_id
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.onnx_export = onnx_export
        self.output_attentions = output_attentions
        self.output_hidden_states = output_hidden_states
        self.use_return_dict = use_return_dict
        self.chunk_size_feed_forward = chunk_size_feed_forward
        for k, v in kwargs.items():
            setattr(self, k, v)

    # -- transformers-style helpers -------------------------------------------------
    @classmethod
    def from_dict(cls, d: Dict[str, Any], **overrides: Any) -> "RecformerConfig":
        d = dict(d)
        d.update(overrides)
        d.pop("model_type", None)
        d.pop("architectures", None)
        return cls(**d)

    @classmethod
    def from_pretrained(cls, name_or_path: str, **overrides: Any) -> "RecformerConfig":
        """Offline resolution: a preset name, a directory holding config.json, or a json file."""
        if name_or_path in _PRESETS:
            return cls.from_dict(_PRESETS[name_or_path], **overrides)
        path = name_or_path
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        if os.path.isfile(path):
            with open(path) as f:
                return cls.from_dict(json.load(f), **overrides)
        raise OSError(
            f"RecformerConfig.from_pretrained: '{name_or_path}' is neither a built-in preset "
            f"({sorted(_PRESETS)}) nor a local config.json (no hub access in this build)"
        )

    def to_dict(self) -> Dict[str, Any]:
        out = copy.deepcopy(self.__dict__)
        out["model_type"] = self.model_type
        return out

    def save_pretrained(self, directory: str) -> None:
        os.makedirs(directory, exist_ok=True)
        with open(os.path.join(directory, "config.json"), "w") as f:
            json.dump(self.to_dict(), f, indent=2, sort_keys=True)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    def window_per_layer(self) -> List[int]:
        w = self.attention_window
        if isinstance(w, int):
            return [w] * self.num_hidden_layers
        return list(w)

    def __repr__(self) -> str:
        return f"RecformerConfig {json.dumps(self.to_dict(), sort_keys=True, default=str)}"
