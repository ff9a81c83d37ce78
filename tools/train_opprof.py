"""Which torch ops issue the C3 step's small elementwise / copy / fill / reduce kernels:
torch.profiler over a few tools/train_bench.py-shaped steps, aten ops by device time with shapes.

    python tools/train_opprof.py [--batch 16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=10000, attention_probs_dropout_prob=0.1))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg)
    model.init_item_embedding(torch.randn(10000, cfg.hidden_size) * 0.5)
    model = model.to(dev).train()
    from recformer_amd.optim import AdamW
    opt = AdamW([p for p in model.parameters() if p.requires_grad], lr=5e-5)
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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=110,
                                                             max_name_column_width=40, max_shapes_column_width=70))


if __name__ == "__main__":
    main()
