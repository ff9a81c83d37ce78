"""C3 finetune-step throughput (BASELINE configs[2]): RecformerForSeqRec forward + backward +
AdamW step under bf16 autocast, 12L/768d, B sequences x L=1024 per step, 10k-item catalog,
full softmax (finetune.sh) or sampled (--negatives k). Dropout 0.1 on hidden layers and on
attention probabilities (the longformer-base config finetune.py loads; --attn-dropout 0 to turn
the latter off).

    python tools/train_bench.py [--batch 16] [--steps 5] [--negatives 0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recformer_amd import RecformerConfig, RecformerForSeqRec  # noqa: E402
from recformer_amd.optim import AdamW  # noqa: E402
from recformer_amd.synth import BASE, synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--negatives", type=int, default=0)
    ap.add_argument("--catalog", type=int, default=10000)
    ap.add_argument("--attn-dropout", type=float, default=0.1)
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16")
    ap.add_argument("--no-dw-split", action="store_true", help="A/B: weight gradients as one GEMM each")
    ap.add_argument("--blas-da", action="store_true", help="A/B: dA of the non-FFN Linears on hipBLASLt")
    ap.add_argument("--no-ffn-fused", action="store_true", help="A/B: FFN as two Linears + torch GELU")
    ap.add_argument("--no-fused-gelu", action="store_true", help="A/B: FFN1 GEMM then F.gelu")
    ap.add_argument("--global-bwd-six", action="store_true", help="A/B: the global backward's six passes over h")
    ap.add_argument("--ab", default=None, help="A/B in one process: alternate blocks of steps with the "
                    "train.py switch of this name True / False and print both medians")
    ap.add_argument("--graph", action="store_true", help="replay the step as one captured HIP graph "
                    "(recformer_amd.graphs.CapturedTrainStep)")
    ap.add_argument("--torch-adamw", action="store_true", help="A/B: torch.optim.AdamW (multi-tensor) instead of "
                    "recformer_amd.optim.AdamW (one HIP launch)")
    ap.add_argument("--ab-knob", default=None, help="A/B in one process: a library knob "
                    "(recformer_amd._lib.set_knob) at 1 / 0, or name=a,b for values a / b")
    ap.add_argument("--global-dh-f32", action="store_true", help="A/B: the global branch's dh as an fp32 product")
    ap.add_argument("--accum", type=int, default=1, help="micro-batches per optimizer step (finetune.py "
                    "gradient_accumulation_steps: loss / k, one optimizer step per k); a timed step = k micro-batches")
    ap.add_argument("--clip", type=float, default=None, help="clip_grad_norm_ before the step (Lightning "
                    "gradient_clip_val=1.0, lightning_pretrain.py:140); with fp16, after scaler.unscale_")
    a = ap.parse_args()
    if a.global_dh_f32:
        from recformer_amd import train
        train.GLOBAL_BWD_DH16 = False
    if a.global_bwd_six:
        from recformer_amd import train
        train.GLOBAL_BWD_MERGED = False
    if a.no_fused_gelu:
        from recformer_amd import train
        train.FUSED_GELU = False
    if a.blas_da:
        from recformer_amd import train
        train.DA_RF_GEMM = False
    if a.no_ffn_fused:
        from recformer_amd import train
        train.FFN_FUSED = False
    if a.no_dw_split:
        from recformer_amd import train
        train.DW_SPLIT_K = False
    dev = torch.device("cuda")
    cfg = RecformerConfig(**dict(BASE, item_num=a.catalog, attention_probs_dropout_prob=a.attn_dropout,
                                 finetune_negative_sample_size=a.negatives))
    torch.manual_seed(0)
    model = RecformerForSeqRec(cfg)
    model.init_item_embedding(torch.randn(a.catalog, cfg.hidden_size) * 0.5)
    model = model.to(dev).train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=5e-5) if a.torch_adamw else AdamW(params, lr=5e-5, capturable=a.graph)
    batch = {k: v.to(dev) for k, v in synth_batch(a.batch, 1024, cfg.vocab_size, seed=7, item_len=21).items()}
    labels = torch.randint(0, a.catalog, (a.batch,), device=dev)

    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    scaler = torch.amp.GradScaler("cuda") if a.dtype == "fp16" else None

    def step():  # one optimizer step: a.accum micro-batches (finetune.py:98-126)
        for _ in range(a.accum):
            with torch.autocast("cuda", dtype=dt):
                loss = model(**batch, labels=labels)
            out = loss / a.accum if a.accum > 1 else loss
            if scaler is not None:  # finetune.py:106-116 (fp16 autocast + GradScaler)
                scaler.scale(out).backward()
            else:
                out.backward()
        if scaler is not None:
            if a.clip is not None:
                scaler.unscale_(opt)
                torch.nn.utils.clip_grad_norm_(params, a.clip, foreach=True)
            scaler.step(opt)
            scaler.update()
        else:
            if a.clip is not None:
                torch.nn.utils.clip_grad_norm_(params, a.clip, foreach=True)
            opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    def set_switch(val):
        """A/B switch: a train.py flag (or models.<flag>) at True / False, or a library knob at 1 / 0
        (name=a,b: values a / b)."""
        from recformer_amd import _lib, models, train
        if a.ab:
            from recformer_amd import graphs as G
            mod, name = ((models, a.ab[len("models."):]) if a.ab.startswith("models.") else
                         (G, a.ab[len("graphs."):]) if a.ab.startswith("graphs.") else (train, a.ab))
            if not hasattr(mod, name):
                raise SystemExit(f"unknown switch {a.ab}")
            setattr(mod, name, val)
            return
        kname, kvals = a.ab_knob, (1, 0)
        if "=" in a.ab_knob:
            kname, v = a.ab_knob.split("=")
            kvals = tuple(int(x) for x in v.split(","))
        _lib.set_knob(kname, kvals[0] if val else kvals[1])

    if a.graph and (a.ab or a.ab_knob):
        # captured A/B: one graph per value of the switch (a library knob's kernel choice is fixed at
        # capture), replays alternated in one process
        from recformer_amd.graphs import CapturedTrainStep
        graphs = {}
        for val in (True, False):
            set_switch(val)
            graphs[val] = CapturedTrainStep(model, opt, dict(batch, labels=labels), autocast_dtype=dt,
                                            warmup=a.warmup, scaler=scaler, accumulation_steps=a.accum,
                                            max_grad_norm=a.clip)
        res = {True: [], False: []}
        for rep in range(6):
            for val in (True, False):
                graphs[val]()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    graphs[val]()
                torch.cuda.synchronize()
                res[val].append((time.perf_counter() - t0) / a.steps * 1e3)
        for val in (True, False):
            v = sorted(res[val])
            print(f"captured {a.ab or a.ab_knob}={val}: ms/step median {v[len(v) // 2]:.2f} min {v[0]:.2f} all "
                  f"{[round(x, 2) for x in res[val]]}")
        return
    if a.graph:
        # fp16 + GradScaler, accumulation and clipping are captured too (device-side inf check / skip /
        # scale update, recformer_amd.graphs.CapturedTrainStep)
        from recformer_amd.graphs import CapturedTrainStep
        captured = CapturedTrainStep(model, opt, dict(batch, labels=labels), autocast_dtype=dt, warmup=a.warmup,
                                     scaler=scaler, accumulation_steps=a.accum, max_grad_norm=a.clip)

        def step():  # noqa: F811 - the captured replays replace the eager step
            for _ in range(a.accum):
                loss = captured()
            return loss
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if a.ab or a.ab_knob:
        # clocks differ across boxes and drift under load: alternate blocks in one process
        res = {True: [], False: []}
        for rep in range(6):
            for val in (True, False):
                set_switch(val)
                step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                torch.cuda.synchronize()
                res[val].append((time.perf_counter() - t0) / a.steps * 1e3)
        for val in (True, False):
            v = sorted(res[val])
            print(f"{a.ab or a.ab_knob}={val}: ms/step median {v[len(v) // 2]:.2f} min {v[0]:.2f} all {[round(x, 2) for x in res[val]]}")
        return
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"workload": f"C3 finetune step (fwd+bwd+AdamW), 12L/768d, L=1024, {a.dtype} autocast, "
                                  f"attention dropout {a.attn_dropout}"
                                  + (", GradScaler" if scaler is not None else "")
                                  + (f", {a.accum} micro-batches per step" if a.accum > 1 else "")
                                  + (f", clip {a.clip}" if a.clip is not None else ""),
                      "batch": a.batch, "accum": a.accum, "negatives": a.negatives, "catalog": a.catalog,
                      "ms_per_step": round(1e3 * el / a.steps, 2),
                      "seq_per_s": round(a.batch * a.accum * a.steps / el, 2),
                      "loss": float(loss.detach()), "optimizer": type(opt).__module__ + ".AdamW", "graph": a.graph,
                      "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}))


if __name__ == "__main__":
    main()
