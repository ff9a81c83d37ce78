"""recformer_amd — MI355X-native (gfx950) Recformer encoder + scorer.

Drop-in for the reference package `recformer` (recformer/__init__.py:1-3): the same class
names and forward() signatures, backed by hand-written HIP kernels in librecformer_hip.so.
"""
from .config import RecformerConfig
from .ranker import Ranker
from .models import (RecformerEmbeddings, RecformerForPretraining, RecformerForSeqRec,
                     RecformerModel, RecformerModelOutput, RecformerPooler,
                     RecformerPretrainingOutput, Similarity, create_position_ids_from_input_ids)

__all__ = [
    "RecformerConfig", "RecformerModel", "RecformerForSeqRec", "RecformerForPretraining",
    "RecformerPretrainingOutput", "RecformerModelOutput", "RecformerEmbeddings", "RecformerPooler",
    "Similarity", "create_position_ids_from_input_ids", "Ranker",
]
