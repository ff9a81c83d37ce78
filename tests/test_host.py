"""Host-side checks that need no GPU: config, drop-in state-dict layout, the C ABI
library exports, and the product path failing loudly without a ROCm device."""
import os
import re

import pytest
import torch

import recformer_amd
from recformer_amd import RecformerConfig, RecformerForPretraining, RecformerForSeqRec, RecformerModel
from recformer_amd import _lib
from tests.common import C1, manifest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_preset_and_roundtrip(tmp_path):
    c = RecformerConfig.from_pretrained("allenai/longformer-base-4096")
    assert (c.hidden_size, c.num_hidden_layers, c.vocab_size, c.max_position_embeddings) == (768, 12, 50265, 4098)
    assert c.layer_norm_eps == 1e-5 and c.pad_token_id == 1 and c.temp == 0.05
    # the attribute writes finetune.py:202-209 performs
    c.max_attr_num, c.max_attr_length, c.max_item_embeddings = 3, 32, 51
    c.attention_window, c.max_token_num, c.item_num = [64] * 12, 1024, 10
    c.save_pretrained(str(tmp_path))
    d = RecformerConfig.from_pretrained(str(tmp_path))
    assert d.to_dict() == c.to_dict()
    with pytest.raises(OSError):
        RecformerConfig.from_pretrained("no/such-model")


@pytest.mark.parametrize("cls", [RecformerModel, RecformerForSeqRec, RecformerForPretraining])
def test_state_dict_layout_matches_reference(cls):
    ref = manifest()["state_dict_layout_C1"][cls.__name__]
    ours = {k: [list(v.shape), str(v.dtype)] for k, v in cls(RecformerConfig(**C1)).state_dict().items()}
    assert ours == ref


def test_reference_checkpoint_loads_strict():
    m = RecformerForSeqRec(RecformerConfig(**C1))
    sd = m.state_dict()
    m2 = RecformerForSeqRec(RecformerConfig(**C1))
    m2.load_state_dict(sd, strict=True)


def _header_functions():
    with open(os.path.join(ROOT, "include", "recformer_hip.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*|const uint64_t\*)\s+(rf_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = _header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, f"{n} declared in the header but not typed in _lib.py"
    assert set(_lib.SIGNATURES) == set(names)
    assert lib.rf_abi_version() == _lib.ABI_VERSION == 2


def test_every_documented_knob_is_readable():
    """The knob names the header documents (rf_debug_set_knob) all resolve, and set / get round-trip;
    an unknown name is an error message, not a crash. Host-side table only (no GPU)."""
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "recformer_hip.h")).read()
    m = re.search(r"knobs? \(([^)]*)\)", hdr.replace("\n *", " "))
    names = re.findall(r'"([a-z0-9_]+)"', m.group(1)) if m else []
    assert "tn_wgs" in names and "gemm_mfma32" in names, names
    for n in names:
        v = _lib.get_knob(n)
        assert _lib.set_knob(n, v) == v and _lib.get_knob(n) == v
    with pytest.raises(_lib.RecformerHipError):
        _lib.get_knob("no_such_knob")


def test_argument_errors_come_back_as_messages():
    lib = _lib.load()
    # bad shape is rejected host-side before any launch (no GPU needed)
    rc = lib.rf_gemm(1, 64, 64, 63, None, 63, None, 63, None, None, 0, None, 64, 0, 0, 0, 1.0, None, None, None)
    assert rc != 0
    assert b"multiple" in lib.rf_last_error()


def test_product_path_has_no_cpu_fallback():
    m = RecformerModel(RecformerConfig(**C1)).eval()
    ids = torch.zeros(1, 64, dtype=torch.long)
    with pytest.raises(_lib.RecformerHipError):
        m(input_ids=ids, item_position_ids=ids)


def test_split_stream_encoding_is_exact():
    """The bf16 path's fp32 residual stream is stored as (hi, lo) 16-bit planes
    (rf_common.h split_f32 / join_f32): restated on the host, every fp32 value - ties,
    negatives, subnormals, exponent carries - decodes exactly, and hi is a bf16 within half an
    ulp of the value (round half-up: differs from round-to-nearest-even only on exact ties)."""
    import torch

    from recformer_amd.ops import join_split
    g = torch.Generator().manual_seed(0)
    v = torch.cat([torch.randn(100000, generator=g) * 10.0 ** torch.randint(-30, 30, (100000,), generator=g),
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 1.00390625, 1.0 + 2 ** -9, -(1.0 + 2 ** -9),
                                 1.9999999, -1.9999999, 1e-40, -1e-40, 3.0e38])])
    u = v.view(torch.int32).long() & 0xFFFFFFFF
    hi = ((u + 0x8000) >> 16) & 0xFFFF
    lo = u & 0xFFFF
    hi_t = hi.to(torch.int32).to(torch.int16).view(torch.bfloat16)
    lo_t = lo.to(torch.int32).to(torch.int16)
    back = join_split(hi_t, lo_t)
    assert torch.equal(back.view(torch.int32), v.view(torch.int32))
    rne = v.to(torch.bfloat16)
    differ = hi_t.view(torch.int16) != rne.view(torch.int16)
    assert (lo[differ] == 0x8000).all()  # only exact ties may round differently


def test_host_library_exports_every_header_symbol():
    from recformer_amd import data
    with open(os.path.join(ROOT, "include", "recformer_host.h")) as f:
        txt = f.read()
    names = sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(rf_\w+)\s*\(", txt, re.M)))
    assert names == ["rf_collate_fill", "rf_collate_lengths", "rf_host_last_error"]
    lib = data.load_host()
    for n in names:
        assert hasattr(lib, n), n


def test_litwrapper_contract():
    """recformer_amd.LitWrapper mirrors litmodels.py: training_step returns outputs.loss,
    validation accuracy = cl_correct_num / cl_total_num, AdamW groups without decay for biases
    and LayerNorm weights, linear warmup schedule stepped per step."""
    from types import SimpleNamespace

    import recformer_amd

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.dense = torch.nn.Linear(4, 4)
            self.LayerNorm = torch.nn.LayerNorm(4)

        def forward(self, x):
            loss = self.LayerNorm(self.dense(x)).pow(2).mean()
            return SimpleNamespace(loss=loss, cl_correct_num=3, cl_total_num=4)

    lit = recformer_amd.LitWrapper(Tiny(), learning_rate=1e-3, warmup_steps=2, weight_decay=0.1, num_training_steps=10)
    loss = lit.training_step({"x": torch.ones(2, 4)}, 0)
    assert loss.requires_grad
    m = lit.validation_step({"x": torch.ones(2, 4)}, 0)
    assert m["accuracy"] == 0.75
    (opt,), (sch,) = lit.configure_optimizers()
    decay, no_decay = opt.param_groups
    assert decay["weight_decay"] == 0.1 and no_decay["weight_decay"] == 0.0
    assert len(decay["params"]) == 1 and len(no_decay["params"]) == 3  # dense.weight | biases, LN.weight
    assert sch["interval"] == "step" and opt.param_groups[0]["lr"] == 0.0  # warmup starts at 0


def test_adamw_host_checks():
    """recformer_amd.optim.AdamW: torch's argument checks, amsgrad refused, and no CPU fallback (a
    CPU parameter raises before any launch)."""
    import pytest
    import torch
    from recformer_amd.optim import AdamW
    p = torch.zeros(3, requires_grad=True)
    with pytest.raises(ValueError):
        AdamW([p], lr=-1.0)
    with pytest.raises(ValueError):
        AdamW([p], betas=(1.0, 0.9))
    with pytest.raises(NotImplementedError):
        AdamW([p], amsgrad=True)
    opt = AdamW([p])
    opt.step()  # no gradient: nothing to do
    p.grad = torch.ones(3)
    with pytest.raises(ValueError):
        opt.step()


def test_package_exports_resolve():
    """Every name in recformer_amd.__all__ resolves (lazy host-side pieces included)."""
    import recformer_amd
    for name in recformer_amd.__all__:
        assert getattr(recformer_amd, name) is not None, name


def test_inputs_embeds_table_and_head_mask_host_logic():
    """inputs_embeds becomes a word table whose rows the token ids index (zero rows up to the padding
    id); head_mask (layers, heads) becomes per-layer context-column scales; the oracle's all-ones mask
    is the identity."""
    from oracle import restatement as R
    from recformer_amd.models import _embeds_as_table, _head_mask_columns
    from tests.common import batch_of, hashed_model, load_golden
    x = torch.randn(2, 5, 8)
    ids, table, pos = _embeds_as_table(x, None, 1)
    assert table.shape == (2 + 10, 8) and not table[:2].any()
    assert torch.equal(table[ids], x)
    assert torch.equal(pos[1], torch.arange(2, 7))
    cfg = RecformerConfig(**C1)
    hm = torch.rand(cfg.num_hidden_layers, cfg.num_attention_heads)
    cols = _head_mask_columns(hm, cfg)
    hd = cfg.hidden_size // cfg.num_attention_heads
    assert cols.shape == (cfg.num_hidden_layers, cfg.hidden_size)
    assert torch.equal(cols[:, ::hd], hm)
    with pytest.raises(ValueError):
        _head_mask_columns(hm[0], cfg)
    g = load_golden("c1_ragged")
    lf = hashed_model(C1, seed=1)
    with torch.no_grad():
        a, _ = R.model_forward(lf.state_dict(), lf.config, **batch_of(g))
        b, _ = R.model_forward(lf.state_dict(), lf.config, **batch_of(g), head_mask=torch.ones_like(hm))
        hz = torch.ones_like(hm)
        hz[0] = 0
        c, _ = R.model_forward(lf.state_dict(), lf.config, **batch_of(g), head_mask=hz)
    assert torch.equal(a, b)
    assert not torch.allclose(a, c)


def test_bench_accounting_of_the_step_as_run():
    """bench.py's algorithmic work per sequence (SURVEY §8d counting) for C2: 176.5 GFLOP with every row
    through the last layer (70.6 us at 2.5 PF dense bf16), 161.8 GFLOP for the CLS-only last layer the
    step runs (64.7 us) — the floors e2e_roofline and model_tflops use; and the CPU baseline carries the
    committed calibration of the restatement against the real reference (within +-15%)."""
    import bench
    full = bench.step_flops_per_seq(1024, 768, 3072, 12, 10000, cls_last=False)
    pruned = bench.step_flops_per_seq(1024, 768, 3072, 12, 10000, cls_last=True)
    assert abs(full["total"] / 1e9 - 176.5) < 0.1 and abs(pruned["total"] / 1e9 - 161.8) < 0.1
    assert pruned["score"] == full["score"] == 2 * 10000 * 768
    assert abs(bench.e2e_floor_us(1024, 768, 3072, 12, 10000, cls_last=False) - 70.6) < 0.05
    assert abs(bench.e2e_floor_us(1024, 768, 3072, 12, 10000, cls_last=True) - 64.72) < 0.05
    cal = bench._cpu_calibration()
    assert cal is not None and cal["within_15pct"] and 0.85 <= cal["port_over_reference"] <= 1.15
    assert os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), cal["file"]))
