"""Which Python lines launch the torch (non-HIP) kernels of the C3 training step.

Runs one eager C3 step (tools/train_bench.py's model, batch and optimizer) under a TorchDispatchMode
that records the Python stack of every aten op on a device tensor and prints, per aten op that
launches a device kernel (fill_/zero_/zeros, add, copy_, index_select, cat, sort, ...), the count per step and the innermost recformer_amd frames that
issued it — the list of torch launches left to fold into the HIP kernels or remove.

    python tools/torch_ops_trace.py [--batch 16]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec  # noqa: E402
from recformer_amd.optim import AdamW  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402

OPS = ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::add", "aten::add_", "aten::copy_",
       "aten::index_select", "aten::index", "aten::cat", "aten::sort", "aten::mul", "aten::mul_", "aten::where",
       "aten::clamp", "aten::sum", "aten::arange", "aten::masked_fill", "aten::to", "aten::_to_copy",
       "aten::index_add_", "aten::index_add", "aten::index_put_", "aten::scatter_add_", "aten::embedding_dense_backward", "aten::div", "aten::neg")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--infer", action="store_true",
                    help="the C2 inference step instead (bench.py: B=64 encode + score, fp32 parameters under autocast)")
    a = ap.parse_args()
    if a.infer:
        a.batch = 64 if a.batch == 16 else a.batch
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

    if a.infer:
        model.eval()

        def step():  # noqa: F811 - bench.py's step
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                return model(**batch)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    # aten-level interception (below autograd, so the engine's own gradient accumulations show up
    # too); the Python stack at dispatch time names the recformer_amd line that issued each op
    per = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    names = {n.split("::")[1] for n in OPS}

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.overloadpacket.__name__
            kw = kwargs or {}
            on_dev = any(torch.is_tensor(x) and x.is_cuda for x in list(args) + list(kw.values()))
            dv = kw.get("device")
            on_dev = on_dev or (dv is not None and torch.device(dv).type == "cuda")
            # every op on (or creating) a device tensor — factories (zeros, full, arange, empty) included
            if on_dev and name not in ("empty", "empty_strided", "view", "_unsafe_view", "t", "transpose",
                                       "slice", "select", "as_strided", "detach", "alias", "expand",
                                       "unsqueeze", "squeeze", "permute", "reshape", "_reshape_alias",
                                       "split", "unbind", "diagonal", "set_", "resize_", "lift_fresh",
                                       "is_same_size", "_local_scalar_dense"):
                st = traceback.extract_stack(limit=40)
                fr = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in st
                      if "recformer_amd" in f.filename or "autograd" in f.filename]
                key = " < ".join(reversed(fr[-a.frames:])) or "(autograd engine)"
                per[name] += 1
                where[name][key] += 1
            return func(*args, **(kwargs or {}))

    with Rec():
        step()
        torch.cuda.synchronize()
    print(f"aten ops on device tensors in one eager {'C2 inference' if a.infer else 'C3'} step (batch {a.batch}): "
          f"{sum(per.values())}")
    for name, n in per.most_common():
        print(f"{n:5d}  {name}")
        for key, m in where[name].most_common(10):
            print(f"         {m:4d}  {key}")


if __name__ == "__main__":
    main()
