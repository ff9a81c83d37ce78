"""Which Python lines launch the torch (non-HIP) kernels of the C3 training step.

Runs one eager C3 step (tools/train_bench.py's model, batch and optimizer) under torch.profiler with
Python stacks and prints, per aten op that launches a device kernel (fill_/zero_/zeros, add, copy_,
index_select, cat, sort, ...), the call count per step and the innermost recformer_amd frames that
issued it — the list of torch launches left to fold into the HIP kernels or remove.

    python tools/torch_ops_trace.py [--batch 16]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec  # noqa: E402
from recformer_amd.optim import AdamW  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402

OPS = ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::add", "aten::add_", "aten::copy_",
       "aten::index_select", "aten::index", "aten::cat", "aten::sort", "aten::mul", "aten::mul_", "aten::where",
       "aten::clamp", "aten::sum", "aten::arange", "aten::masked_fill", "aten::to", "aten::_to_copy",
       "aten::index_add_", "aten::scatter_add_", "aten::embedding_dense_backward", "aten::div", "aten::neg")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000, finetune_negative_sample_size=0))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg)
    model.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    model = model.to(dev).train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = AdamW(params, lr=5e-5)
    batch = {k: v.to(dev) for k, v in synth_batch(a.batch, 1024, cfg.vocab_size, seed=7, item_len=21).items()}
    labels = torch.randint(0, 10000, (a.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = model(**batch, labels=labels)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        step()
        torch.cuda.synchronize()
    per = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        # only the outermost aten op of a chain (a zeros that calls fill_ counts once)
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue
        frames = [f for f in (ev.stack or []) if "recformer_amd" in f or "torch/autograd" in f]
        key = " < ".join(f.split("/")[-1] for f in frames[:a.frames]) or "(no recformer_amd frame)"
        per[ev.name] += 1
        where[ev.name][key] += 1
    print(f"torch ops in one eager C3 step (batch {a.batch}): {sum(per.values())}")
    for name, n in per.most_common():
        print(f"{n:5d}  {name}")
        for key, m in where[name].most_common(8):
            print(f"         {m:4d}  {key}")


if __name__ == "__main__":
    main()
