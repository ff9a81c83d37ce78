"""One rank of the world-2 C4 pretraining check (tests/test_gpu_pretrain.py::test_c4_pretrain_dp_world2).

Run as `python -m tests._pretrain_dp_worker OUTDIR MODE` with RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set. Both ranks share GPU 0; the process group is gloo (RCCL needs one rank per device).
Each rank runs RecformerForPretraining (12L/768d, the c4_pretrain fixture's weights) on its row of the
fixture batch: forward (z all-gathered across the ranks, models.py:474-490), backward with
dp.GradBucketer launching the bucket all-reduces from the gradient hooks, finish(); then writes its
loss, cl_correct_num, the collective count and, per parameter, the averaged gradient's norm and its
entries at the fixture's slice positions to OUTDIR/rank{r}.npz.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def main():
    outdir, mode = sys.argv[1], sys.argv[2]
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from recformer_amd import dp
        from tests.test_gpu_pretrain import ALIAS, FIX, _ctx, build_model, fixture_inputs
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        gz = np.load(FIX)
        m = build_model(dev)
        b = dp.GradBucketer(m.parameters(), bucket_bytes=64 << 20)
        batch = {k: v.to(dev) for k, v in fixture_inputs(gz, slice(rank, rank + 1)).items()}
        with _ctx(mode):
            out = m(**batch)
        out.loss.backward()
        n = b.finish()
        params = dict(m.named_parameters())
        arrays = {"loss": np.asarray(float(out.loss)), "correct": np.asarray(int(out.cl_correct_num)),
                  "collectives": np.asarray(n), "nbuckets": np.asarray(len(b.buckets))}
        for name in (str(x) for x in gz["names"]):
            g = params[ALIAS.get(name, name)].grad.detach().double().flatten()
            arrays[f"{name}:norm"] = np.asarray(float(g.norm()))
            arrays[f"{name}:val"] = g[torch.from_numpy(gz[f"g:{name}:pos"]).to(dev)].cpu().numpy()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **arrays)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
