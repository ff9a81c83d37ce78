"""recformer_amd.optim.AdamW (one rf_adamw_step launch per step) against torch.optim.AdamW, the
optimizer of every reference driver (optimization.py:28-32, litmodels.py:42-56)."""
import pytest
import torch

from recformer_amd.optim import AdamW

pytestmark = pytest.mark.gpu

SHAPES = [(1,), (3,), (768,), (1000, 3), (8197,), (2304, 768), (3, 5, 7), (20000, 768)]


def _params(dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.randn(s, generator=g).to(dev).requires_grad_(True) for s in SHAPES]


def _groups(ps, wd):
    return [{"params": ps[::2], "weight_decay": wd}, {"params": ps[1::2], "weight_decay": 0.0}]


@pytest.mark.parametrize("kw", [dict(lr=5e-5, wd=0.01), dict(lr=1e-3, wd=0.1, betas=(0.8, 0.95), eps=1e-6),
                                dict(lr=2e-4, wd=0.0, maximize=True), dict(lr=1e-3, wd=0.01, betas=(0.3, 0.9))])
def test_adamw_matches_torch(dev, kw):
    """Six steps over tensors of 1 .. 15M elements (sizes not multiples of 4 or of the 8192-element
    workgroup chunk, two parameter groups with and without weight decay), a parameter without a
    gradient in step 3 (skipped, its step count not advanced, as torch), beta1 above and below the
    lerp formula's 0.5 switch; parameters and both moments agree with torch's AdamW to fp32 rounding
    and the state_dict loads into torch's AdamW."""
    kw = dict(kw)
    wd = kw.pop("wd")
    a, b = _params(dev), _params(dev)
    oa = AdamW(_groups(a, wd), **kw)
    ob = torch.optim.AdamW(_groups(b, wd), foreach=True, **kw)
    g = torch.Generator(device="cpu").manual_seed(1)
    for step in range(6):
        grads = [torch.randn(p.shape, generator=g).to(dev) * (1 + i) for i, p in enumerate(a)]
        for ps in (a, b):
            for i, p in enumerate(ps):
                p.grad = None if (step == 2 and i == 3) else grads[i].clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, rtol=2e-6, atol=2e-7), float((pa - pb).abs().max())
        sa, sb = oa.state[pa], ob.state[pb]
        assert float(sa["step"]) == float(sb["step"])
        assert torch.allclose(sa["exp_avg"], sb["exp_avg"], rtol=1e-6, atol=1e-7)
        assert torch.allclose(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-6, atol=1e-9)
    assert float(oa.state[a[3]]["step"]) == 5.0
    oc = torch.optim.AdamW(_groups(b, wd), **kw)
    oc.load_state_dict(oa.state_dict())
    assert float(oc.state[b[0]]["step"]) == 6.0


def test_adamw_gradscaler_skips_inf_step(dev):
    """fp16 GradScaler (finetune.py:116-126): grads unscaled by the scaler, a step with an inf
    gradient skipped (parameters, moments and step counts unchanged), the next finite step taken
    exactly as torch's AdamW under the same scaler."""
    a, b = _params(dev)[:4], _params(dev)[:4]
    oa, ob = AdamW(a, lr=1e-3), torch.optim.AdamW(b, lr=1e-3)
    sa, sb = torch.amp.GradScaler("cuda", init_scale=1024.0), torch.amp.GradScaler("cuda", init_scale=1024.0)
    for step in range(3):
        for ps, opt, sc in ((a, oa, sa), (b, ob, sb)):
            loss = sum((p * (i + 1)).sum() for i, p in enumerate(ps))
            sc.scale(loss).backward()
            if step == 1:
                ps[2].grad[0] = float("inf")
            before = [p.detach().clone() for p in ps]
            sc.step(opt)
            sc.update()
            opt.zero_grad(set_to_none=True)
            if step == 1:
                assert all(torch.equal(x, p) for x, p in zip(before, ps))
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, rtol=2e-6, atol=2e-7)
        assert float(oa.state[pa]["step"]) == float(ob.state[pb]["step"]) == 2.0


def test_adamw_rejects_unsupported(dev):
    p = torch.zeros(4, 4, device=dev, requires_grad=True)
    p.grad = torch.zeros(4, 4, device=dev).t()
    with pytest.raises(ValueError):
        AdamW([p]).step()
    q = torch.zeros(4, device=dev, dtype=torch.float16, requires_grad=True)
    q.grad = torch.zeros_like(q)
    with pytest.raises(ValueError):
        AdamW([q]).step()
