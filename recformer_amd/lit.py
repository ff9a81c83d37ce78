"""LitWrapper (recformer/litmodels.py:7-64): the pretraining module wrapper, same constructor,
hooks and optimizer grouping. A pytorch_lightning.LightningModule when Lightning is installed
(lightning_pretrain.py drives it unchanged); otherwise a plain nn.Module with the same methods,
for the build's own DP driver (recformer_amd/dp.py) or a hand-written loop."""
from __future__ import annotations

import torch
import torch.nn as nn
from .optim import AdamW

try:  # Lightning is not in this image; the wrapper keeps its contract either way
    import pytorch_lightning as _pl
    _Base = _pl.LightningModule
except Exception:  # pragma: no cover - depends on the environment
    _pl = None
    _Base = nn.Module


class LitWrapper(_Base):
    def __init__(self, model: nn.Module, learning_rate: float = 5e-5, warmup_steps: int = 0,
                 weight_decay: float = 0.0, num_training_steps: int = 0):
        super().__init__()
        if _pl is not None:
            self.save_hyperparameters(ignore=["model"])
        self.learning_rate = learning_rate
        self.warmup_steps = warmup_steps
        self.weight_decay = weight_decay
        self.num_training_steps = num_training_steps  # Lightning: trainer.estimated_stepping_batches
        self.model = model
        self.logged = {}

    def forward(self, **inputs):
        return self.model(**inputs)

    def training_step(self, batch, batch_idx):
        return self(**batch).loss  # litmodels.py:25-28

    def validation_step(self, batch, batch_idx):
        outputs = self(**batch)  # litmodels.py:30-40
        total = outputs.cl_total_num
        accuracy = outputs.cl_correct_num / total if total > 0 else 0.0
        metrics = {"val_loss": outputs.loss, "accuracy": accuracy}
        if _pl is not None:
            self.log_dict(metrics, on_epoch=True, prog_bar=True)
        else:
            self.logged = metrics
        return metrics

    def configure_optimizers(self):
        """litmodels.py:42-64: AdamW, no decay on biases and LayerNorm weights, linear warmup/decay
        schedule stepped per optimizer step."""
        from transformers import get_linear_schedule_with_warmup
        no_decay = ["bias", "LayerNorm.weight"]
        named = list(self.model.named_parameters())
        groups = [
            {"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": self.weight_decay},
            {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0},
        ]
        # recformer_amd.optim.AdamW: torch's AdamW update, state_dict and GradScaler behaviour, one HIP launch
        optimizer = AdamW(groups, lr=self.learning_rate)
        total = (self.trainer.estimated_stepping_batches if _pl is not None and getattr(self, "_trainer", None)
                 else self.num_training_steps)
        scheduler = get_linear_schedule_with_warmup(optimizer, num_warmup_steps=self.warmup_steps,
                                                    num_training_steps=total)
        return [optimizer], [{"scheduler": scheduler, "interval": "step", "frequency": 1}]
