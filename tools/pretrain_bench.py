"""C4 pretraining-step throughput (BASELINE configs[3]): RecformerForPretraining (two views,
MLM on both, item-item contrastive with the z all-gather across ranks, models.py:382-520) forward +
backward + bucketed RCCL gradient all-reduce overlapped with it (recformer_amd.dp.GradBucketer) + AdamW, bf16
autocast, 12L/768d. Per rank B sequences: view a = a 1024-token item prefix, view b = one item
(<s> + 96 tokens -> 128), 15% of the tokens masked (mask id 50264, labels elsewhere -100).

    python tools/pretrain_bench.py [--batch 4] [--steps 5]            (one GPU)
    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/pretrain_bench.py   (DP over N GPUs)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForPretraining, dp  # noqa: E402
from recformer_amd.optim import AdamW  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def view(B, L, vocab, seed, item_len, mask_id, g):
    b = synth_batch(B, L, vocab, seed=seed, item_len=item_len)
    ids = b["input_ids"]
    m = (torch.rand(ids.shape, generator=g) < 0.15) & (b["attention_mask"] > 0)
    m[:, 0] = False
    labels = torch.where(m, ids, torch.full_like(ids, -100))
    mlm_ids = torch.where(m, torch.full_like(ids, mask_id), ids)
    return b, mlm_ids, labels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4, help="sequences per rank per step")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--len-a", type=int, default=1024)
    ap.add_argument("--len-b", type=int, default=128)
    ap.add_argument("--no-share-casts", action="store_true", help="A/B: per-pass weight casts")
    ap.add_argument("--autograd-global-bwd", action="store_true", help="A/B: global rows' backward by autograd")
    ap.add_argument("--graph", action="store_true", help="replay the step as one captured HIP graph (any world "
                    "size: the bucketed all-reduce is captured with the backward)")
    ap.add_argument("--torch-adamw", action="store_true", help="A/B: torch.optim.AdamW instead of the HIP AdamW")
    ap.add_argument("--full-lm-head", action="store_true", help="A/B: LM head over every token")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16", "fp16"], default="bf16",
                    help="gradient exchange on the wire (dp.GradBucketer comm_dtype; bf16/fp16 = 16-bit, "
                         "as DeepSpeed precision=16)")
    a = ap.parse_args()
    if a.full_lm_head:
        from recformer_amd import models
        models.LM_HEAD_MASKED_ONLY = False
    if a.no_share_casts:
        from recformer_amd import models
        models.SHARE_TRAIN_CASTS = False
    if a.autograd_global_bwd:
        from recformer_amd import train
        train.GLOBAL_BWD_CLOSED_FORM = False
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    cfg = RecformerConfig(**dict(BASE, attention_probs_dropout_prob=0.0))
    torch.manual_seed(0)
    model = RecformerForPretraining(cfg).to(dev).train()
    opt = torch.optim.AdamW(model.parameters(), lr=5e-5) if a.torch_adamw else AdamW(model.parameters(), lr=5e-5,
                                                                                        capturable=a.graph)
    g = torch.Generator().manual_seed(100 + rank)
    va, mlm_a, lab_a = view(a.batch, a.len_a, cfg.vocab_size, 10 + rank, 21, cfg.vocab_size - 1, g)
    vb, mlm_b, lab_b = view(a.batch, a.len_b, cfg.vocab_size, 20 + rank, 96, cfg.vocab_size - 1, g)
    batch = {f"{k}_a": v for k, v in va.items()}
    batch.update({f"{k}_b": v for k, v in vb.items()})
    batch.update(mlm_input_ids_a=mlm_a, mlm_labels_a=lab_a, mlm_input_ids_b=mlm_b, mlm_labels_b=lab_b)
    batch = {k: v.to(dev) for k, v in batch.items()}

    wire = {"fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}[a.comm_dtype]
    bucketer = dp.GradBucketer(model.parameters(), comm_dtype=wire) if world > 1 else None

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(**batch)
        out.loss.backward()
        if bucketer is not None:  # buckets were launched during backward; wait + average
            bucketer.finish()
        opt.step()
        if bucketer is not None:
            bucketer.zero_grad()  # the bucket views stay the gradients
        else:
            opt.zero_grad(set_to_none=True)
        return out

    if a.graph:
        # the bucketed RCCL all-reduces run inside the graph (launched from the backward hooks during
        # capture, recorded with the backward they overlap); cl_correct_num from the captured output
        from recformer_amd.graphs import CapturedTrainStep
        captured = CapturedTrainStep(model, opt, batch, warmup=a.warmup, bucketer=bucketer)

        class _Out:
            pass

        def step():  # noqa: F811 - the captured replay replaces the eager step
            o = _Out()
            o.loss = captured()
            o.cl_correct_num = captured.output.cl_correct_num
            return o
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = dp.max_over_ranks(time.perf_counter() - t0, device=dev)
    if rank == 0:
        print(json.dumps({"workload": "C4 pretrain step (4 encoder passes, MLM + contrastive, grad all-reduce, AdamW), "
                                      "12L/768d, bf16 autocast",
                          "n_gpus": world, "batch_per_rank": a.batch, "len_a": a.len_a, "len_b": a.len_b,
                          "ms_per_step": round(1e3 * dt / a.steps, 2),
                          "seq_per_s": round(world * a.batch * a.steps / dt, 2),
                          "loss": float(out.loss.detach()), "cl_correct": int(out.cl_correct_num), "graph": a.graph,
                          "grad_wire": a.comm_dtype if bucketer is not None else None,
                          "wire_mb_per_step": (round(bucketer.bucket_bytes_on_wire() / 1e6, 1)
                                               if bucketer is not None else None),
                          "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
