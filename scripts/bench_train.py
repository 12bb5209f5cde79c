"""Training-step throughput of the native path (3DPW,
T=40, V=23, 32 sequences per GPU per step; also a large-batch variant).

One step = PredictionEngine.train's body (engine/prediction.py:231-294):
train-mode forward of the batch and of its time reversal, two mpjpe losses,
native backward, Adam.  Prints one JSON line per batch size.

  python scripts/bench_train.py [--batch 32 256] [--steps 20] [--warmup 5]
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

from engine import mpjpe_error_3d  # noqa: E402
from model import get_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[32, 256])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                 joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    for B in a.batch:
        torch.manual_seed(0)
        m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
        m._dstd_inplace_grads = True  # what engine.PredictionEngine.train opts into (prediction.py:161)
        opt = torch.optim.Adam(m.parameters(), lr=3e-3)
        g = torch.Generator().manual_seed(1234)
        seq = torch.randn(B, 40, 69, generator=g)
        inp = seq.clone()
        inp[:, 10:] = inp[:, 9:10]
        inv = seq.flip(1).clone()
        inv[:, 10:] = inv[:, 9:10]
        seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
        seq_inv = seq.flip(1).contiguous()

        def step():
            out = m(inp.view(B, 40, 23, 3)).view(B, 40, 69)
            out_i = m(inv.view(B, 40, 23, 3)).view(B, 40, 69)
            loss = (mpjpe_error_3d(out, seq) + mpjpe_error_3d(out_i, seq_inv)) / 2
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(a.steps):
            loss = step()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        ms = e0.elapsed_time(e1) / a.steps
        print(json.dumps({"metric": "train_sequences_per_sec", "value": round(B / ms * 1e3, 1),
                          "unit": "sequences/s", "ms_per_step": round(ms, 3), "host_ms_per_step": round(wall, 3),
                          "batch": B, "steps": a.steps, "dtype": "f32", "loss": round(float(loss), 4),
                          "config": {"workload": "3dpw T=40 V=23, 2 fwd + 1 bwd + Adam", "inverse": True}}),
              flush=True)


if __name__ == "__main__":
    main()
