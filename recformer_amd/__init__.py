"""recformer_amd — MI355X-native (gfx950) Recformer encoder + scorer.

Drop-in for the reference package `recformer` (recformer/__init__.py:1-3): the same class
names and forward() signatures, backed by hand-written HIP kernels in librecformer_hip.so.
"""
from .config import RecformerConfig
from .ranker import CatalogShard, Ranker, rank_catalog, retrieve
from .models import (RecformerEmbeddings, RecformerForPretraining, RecformerForSeqRec,
                     RecformerModel, RecformerModelOutput, RecformerPooler,
                     RecformerPretrainingOutput, Similarity, create_position_ids_from_input_ids)

_LAZY = {"RecformerTokenizer": "data", "FinetuneDataCollatorWithPadding": "data",
         "EvalDataCollatorWithPadding": "data", "LitWrapper": "lit", "GraphedForward": "graphs",
         "CapturedTrainStep": "graphs", "AdamW": "optim"}


def __getattr__(name):  # host-side pieces load transformers / the host library on first use
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module(f".{_LAZY[name]}", __name__), name)
    raise AttributeError(name)


__all__ = [
    "RecformerConfig", "RecformerModel", "RecformerForSeqRec", "RecformerForPretraining",
    "RecformerPretrainingOutput", "RecformerModelOutput", "RecformerEmbeddings", "RecformerPooler",
    "Similarity", "create_position_ids_from_input_ids", "Ranker", "rank_catalog", "CatalogShard", "retrieve", "RecformerTokenizer",
    "FinetuneDataCollatorWithPadding", "EvalDataCollatorWithPadding", "LitWrapper", "GraphedForward",
    "CapturedTrainStep", "AdamW",
]
