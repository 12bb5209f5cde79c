"""Where the host time of bench.train_leg's eager B=32 step goes: per phase
(forward pair, losses, zero_grad, backward, Adam) host time without syncs,
and each phase's device time (events on the current stream).  Prints one
JSON line per variant."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
from engine import mpjpe_error_3d  # noqa: E402
from model import get_model  # noqa: E402


def run(B=32, steps=30, warmup=5, **adam_kw):
    dev = torch.device("cuda", 0)
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    torch.manual_seed(0)
    m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
    m._dstd_inplace_grads = True
    opt = torch.optim.Adam(m.parameters(), lr=3e-3, **adam_kw)
    g = torch.Generator().manual_seed(1234)
    seq = torch.randn(B, 40, 69, generator=g)
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]
    inv = seq.flip(1).clone()
    inv[:, 10:] = inv[:, 9:10]
    seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
    seq_inv = seq.flip(1).contiguous()
    names = ["fwd", "loss", "zero", "bwd", "adam"]
    host = {k: 0.0 for k in names}
    gpu = {k: 0.0 for k in names}
    for it in range(warmup + steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        hs = []
        ev[0].record()
        hs.append(time.perf_counter())
        out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
        ev[1].record()
        hs.append(time.perf_counter())
        loss = (mpjpe_error_3d(out.reshape(B, 40, 69), seq) + mpjpe_error_3d(out_i.reshape(B, 40, 69), seq_inv)) / 2
        ev[2].record()
        hs.append(time.perf_counter())
        opt.zero_grad()
        ev[3].record()
        hs.append(time.perf_counter())
        loss.backward()
        ev[4].record()
        hs.append(time.perf_counter())
        opt.step()
        ev[5].record()
        hs.append(time.perf_counter())
        torch.cuda.synchronize()
        if it >= warmup:
            for i, k in enumerate(names):
                host[k] += (hs[i + 1] - hs[i]) * 1e6 / steps
                gpu[k] += ev[i].elapsed_time(ev[i + 1]) * 1e3 / steps
    return {"adam": adam_kw or "default", "host_us": {k: round(v, 1) for k, v in host.items()},
            "host_total_us": round(sum(host.values()), 1),
            "event_us": {k: round(v, 1) for k, v in gpu.items()}, "event_total_us": round(sum(gpu.values()), 1)}


if __name__ == "__main__":
    for kw in ({}, {"foreach": True}, {"fused": True}):
        print(json.dumps(run(**kw)), flush=True)
