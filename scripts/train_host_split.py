"""Host time of the native calls inside one B=32 training step (idle queue):
the model forward / backward C calls (dstd_model_train_{fwd,bwd}) timed on
the host around the ctypes call itself, against the whole step's phases
(scripts/train_host_probe.py) -- how much of the step's host time is the
library's launch sequence and how much torch / autograd / Python."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
import dstd_native as native  # noqa: E402
from engine import mpjpe_error_3d  # noqa: E402
from model import get_model  # noqa: E402
import model.dstdgcn as MD  # noqa: E402

acc = {"fwd_c": 0.0, "bwd_c": 0.0}
L = native.lib()
for name in ("dstd_model_train_fwd_ex", "dstd_model_train_bwd_ex"):
    fn = getattr(L, name)

    class Timed:
        def __init__(self, fn, key):
            self.fn, self.key = fn, key

        def __call__(self, *a):
            t0 = time.perf_counter()
            r = self.fn(*a)
            acc[self.key] += time.perf_counter() - t0
            return r
    setattr(L, name, Timed(fn, "fwd_c" if "fwd" in name else "bwd_c"))

# the autograd Function's backward as a whole (Python + the C call)
_orig_bwd = MD._ModelTrain.backward


def _timed_bwd(ctx, dy):
    t0 = time.perf_counter()
    r = _orig_bwd(ctx, dy)
    acc["bwd_fn"] += time.perf_counter() - t0
    return r


MD._ModelTrain.backward = staticmethod(_timed_bwd)
acc["bwd_fn"] = 0.0
ph = {"fwd": 0.0, "loss": 0.0, "zero": 0.0, "bwd": 0.0, "adam": 0.0}
B, steps = 32, 20
dev = torch.device("cuda", 0)
opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
            joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
torch.manual_seed(0)
m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
m._dstd_inplace_grads = True
opt = torch.optim.Adam(m.parameters(), lr=3e-3, fused=True)
g = torch.Generator().manual_seed(1234)
seq = torch.randn(B, 40, 69, generator=g)
inp = seq.clone()
inp[:, 10:] = inp[:, 9:10]
inv = seq.flip(1).clone()
inv[:, 10:] = inv[:, 9:10]
seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
seq_inv = seq.flip(1).contiguous()
tot = 0.0
for it in range(5 + steps):
    if it == 5:
        acc.update(dict.fromkeys(acc, 0.0))
        tot = 0.0
    torch.cuda.synchronize()
    if it == 5:
        ph = dict.fromkeys(ph, 0.0)
    t = [time.perf_counter()]
    out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
    t.append(time.perf_counter())
    loss = (mpjpe_error_3d(out.reshape(B, 40, 69), seq) + mpjpe_error_3d(out_i.reshape(B, 40, 69), seq_inv)) / 2
    t.append(time.perf_counter())
    opt.zero_grad()
    t.append(time.perf_counter())
    loss.backward()
    t.append(time.perf_counter())
    opt.step()
    t.append(time.perf_counter())
    for k, a, b in zip(ph, t, t[1:]):
        ph[k] += b - a
    tot += t[-1] - t[0]
torch.cuda.synchronize()
print(json.dumps({"step_host_us": round(tot / steps * 1e6, 1),
                  "phases_us": {k: round(v / steps * 1e6, 1) for k, v in ph.items()},
                  "fwd_c_call_us": round(acc["fwd_c"] / steps * 1e6, 1),
                  "bwd_function_us": round(acc["bwd_fn"] / steps * 1e6, 1),
                  "bwd_c_call_us": round(acc["bwd_c"] / steps * 1e6, 1)}))
