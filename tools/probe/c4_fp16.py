"""Probe: C4 fp16-autocast gradient cosines vs the fixture with training-path switches toggled."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from recformer_amd import models, train  # noqa: E402
from tests.test_gpu_pretrain import ALIAS, FIX, build_model, fixture_inputs, _zero_grad_param  # noqa: E402


def run(tag, dt):
    gz = np.load(FIX)
    dev = torch.device("cuda")
    m = build_model(dev)
    batch = {k: v.to(dev) for k, v in fixture_inputs(gz).items()}
    with torch.autocast("cuda", dtype=dt):
        out = m(**batch)
    out.loss.backward()
    params = dict(m.named_parameters())
    worst = []
    for n in (str(x) for x in gz["names"]):
        if _zero_grad_param(n):
            continue
        gr = params[ALIAS.get(n, n)].grad.detach().double().flatten()
        got = gr[torch.from_numpy(gz[f"g:{n}:pos"]).to(dev)].float().cpu()
        ref = torch.from_numpy(gz[f"g:{n}:val"])
        worst.append((F.cosine_similarity(got.reshape(1, -1), ref.reshape(1, -1)).item(), n))
    worst.sort()
    print(tag, dt, "loss", float(out.loss), "worst", [(round(c, 4), n) for c, n in worst[:4]], flush=True)


for dt in (torch.float16, torch.bfloat16):
    run("default", dt)
    train.DW_HIP = False
    run("DW_HIP=0", dt)
    train.DW_HIP = True
    models.LM_HEAD_HIP = False
    run("LM_HEAD_HIP=0", dt)
    models.LM_HEAD_HIP = True
    train.EMBED_BWD_HIP = False
    run("EMBED=0", dt)
    train.EMBED_BWD_HIP = True
