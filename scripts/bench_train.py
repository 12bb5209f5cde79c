"""Training-step throughput of the native path (3DPW,
T=40, V=23, 32 sequences per GPU per step; also a large-batch variant).

One step = PredictionEngine.train's body (engine/prediction.py:231-294):
train-mode forward of the batch and of its time reversal (as the engine runs
it: one DSTDGCN.forward_pair, per-half BatchNorm statistics; --two-calls for
two separate forwards), two mpjpe losses, native backward, Adam.  Prints one
JSON line per batch size.

  python scripts/bench_train.py [--batch 32 256] [--steps 20] [--warmup 5]

Data parallel (32 sequences per GPU on 8 GPUs), one
process per GPU over RCCL, the engine's step (dstd_dist: weights broadcast
once, one flat all-reduce of the gradient arena per step before Adam);
the time is the max over ranks, the value the sequences of all ranks:

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      scripts/bench_train.py --batch 32
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dstd-gcn_amd")):
    sys.path.insert(0, p)

import dstd_dist  # noqa: E402
from engine import mpjpe_error_3d  # noqa: E402
from model import get_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[32, 256])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--two-calls", action="store_true", help="two model calls instead of forward_pair")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 or "LOCAL_RANK" in os.environ:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", torch.cuda.current_device())
    distributed = torch.distributed.is_available() and torch.distributed.is_initialized()
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                 joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    for B in a.batch:
        torch.manual_seed(0)
        m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
        m._dstd_inplace_grads = True  # what engine.PredictionEngine.train opts into (prediction.py:161)
        opt = torch.optim.Adam(m.parameters(), lr=3e-3, fused=True)  # the engine's optimizer (prediction.py:166)
        if distributed:
            dstd_dist.broadcast_module(m)
        g = torch.Generator().manual_seed(1234 + rank)  # each rank its own shard of sequences
        seq = torch.randn(B, 40, 69, generator=g)
        inp = seq.clone()
        inp[:, 10:] = inp[:, 9:10]
        inv = seq.flip(1).clone()
        inv[:, 10:] = inv[:, 9:10]
        seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
        seq_inv = seq.flip(1).contiguous()

        def step():
            if a.two_calls:
                out, out_i = m(inp.view(B, 40, 23, 3)), m(inv.view(B, 40, 23, 3))
            else:
                out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
            out, out_i = out.reshape(B, 40, 69), out_i.reshape(B, 40, 69)
            loss = (mpjpe_error_3d(out, seq) + mpjpe_error_3d(out_i, seq_inv)) / 2
            opt.zero_grad()
            loss.backward()
            if distributed:
                dstd_dist.allreduce_grads(m.parameters())
            opt.step()
            return loss

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if distributed:
            torch.distributed.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(a.steps):
            loss = step()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        ms = e0.elapsed_time(e1) / a.steps
        if distributed:  # the slowest rank sets the step
            t = torch.tensor([ms, wall], device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            ms, wall = float(t[0]), float(t[1])
        if rank == 0:
            print(json.dumps({"metric": "train_sequences_per_sec", "value": round(world * B / ms * 1e3, 1),
                              "unit": "sequences/s", "ms_per_step": round(ms, 3), "host_ms_per_step": round(wall, 3),
                              "batch": B, "n_gpus": world, "steps": a.steps, "dtype": "f32",
                              "loss": round(float(loss.detach()), 4), "scaling": "weak",
                              "config": {"workload": "3dpw T=40 V=23, 2 fwd + 1 bwd + Adam", "inverse": True,
                                         "forward": "two calls" if a.two_calls else "forward_pair",
                                         "parallelism": f"dp{world}"}}),
                  flush=True)
    if distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
