"""Load the REAL reference `recformer/models.py` in this build container (test infrastructure).

ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product package. Used by
`oracle/gen_golden.py` to produce `tests/golden/*.npz` and to pin the CPU restatement
(`oracle/restatement.py`) against the reference itself. It does not exist on the GPU
box (`/root/reference` is absent there); nothing on the box imports this file.

`import recformer` fails here (recformer/__init__.py:3 -> litmodels.py:3 imports
pytorch_lightning, which is not installed), so `recformer/models.py` is loaded by
file path. Three runtime shims bridge transformers 4.28 (pinned, requirements.txt:3)
-> 5.15 (installed) API breaks; no reference file is modified:
  1. RecformerConfig's positional super().__init__ (models.py:40) vs the keyword-only
     LongformerConfig: we build a LongformerConfig(**kw) and set the 10 Recformer
     fields (models.py:43-55) on it.
  2. get_extended_attention_mask(mask, shape, device) (models.py:327): 5.x reads the
     3rd arg as dtype. Patched with the 4.28 body (1 - m) * finfo(dtype).min.
  3. LongformerEncoder.forward no longer takes head_mask (models.py:337): dropped
     (every caller passes None).
"""
from __future__ import annotations

import importlib.util
import sys

sys.dont_write_bytecode = True  # never write .pyc into /root/reference

REF_ROOT = "/root/reference"

_MOD = None


def load_reference_models():
    global _MOD
    if _MOD is not None:
        return _MOD
    import torch
    from transformers.models.longformer import modeling_longformer as TF

    spec = importlib.util.spec_from_file_location(
        "_ref_recformer_models", f"{REF_ROOT}/recformer/models.py"
    )
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)

    # shim 2: 4.28 semantics of get_extended_attention_mask
    def _ext_mask(self, attention_mask, input_shape, device=None, dtype=None):
        dt = self.dtype
        m = attention_mask[:, None, None, :].to(dt)
        return (1.0 - m) * torch.finfo(dt).min

    mod.RecformerModel.get_extended_attention_mask = _ext_mask

    # shim 3: drop head_mask
    if not getattr(TF.LongformerEncoder, "_rf_shim", False):
        orig = TF.LongformerEncoder.forward

        def _enc_forward(self, hidden_states, attention_mask=None, head_mask=None, **kw):
            assert head_mask is None
            return orig(self, hidden_states, attention_mask=attention_mask, **kw)

        TF.LongformerEncoder.forward = _enc_forward
        TF.LongformerEncoder._rf_shim = True
    _MOD = mod
    return mod


_RECFORMER_FIELDS = dict(
    token_type_size=4,
    max_token_num=2048,
    max_item_embeddings=32,
    max_attr_num=12,
    max_attr_length=8,
    pooler_type="cls",
    temp=0.05,
    mlm_weight=0.1,
    item_num=0,
    finetune_negative_sample_size=0,
)


def make_reference_config(**kw):
    """shim 1: a LongformerConfig carrying the Recformer attributes."""
    from transformers import LongformerConfig

    rec = dict(_RECFORMER_FIELDS)
    for k in list(kw):
        if k in rec:
            rec[k] = kw.pop(k)
    cfg = LongformerConfig(**kw)
    for k, v in rec.items():
        setattr(cfg, k, v)
    return cfg
