"""Per-tensor gradient error of the native training step vs the reference's
fp64 gradients (train_grads.npz), next to the error of two other fp32
implementations (the reference's own fp32 run and the CPU oracle in fp32).
Diagnostic for tests/test_gpu_train.py; prints a sorted table."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from conftest import group, load_npz  # noqa: E402
from oracle import dstdgcn_oracle as O  # noqa: E402
from test_gpu_train import _model_3dpw  # noqa: E402
from engine import mpjpe_error_3d  # noqa: E402

m, d = _model_3dpw()
g = load_npz("train_grads.npz")
inp, inv, seq = (torch.from_numpy(d[f"train/{n}0"]).cuda() for n in ("inp", "inv", "seq"))
B, T, VC = inp.shape
out = m(inp.view(B, T, 23, 3)).view(B, T, VC)
out_i = m(inv.view(B, T, 23, 3)).view(B, T, VC)
((mpjpe_error_3d(out, seq) + mpjpe_error_3d(out_i, seq.flip(1))) / 2).backward()
P = O.train_params(group(d, "train/sd0/"), torch.float32)
_, l32 = O.step_loss(P, tuple(d[f"train/{n}0"] for n in ("inp", "inv", "seq")), 5)
l32.backward()
named = dict(m.named_parameters())
rows = []
for k in [k[4:] for k in g.files if k.startswith("g64/")]:
    ref = g["g64/" + k]
    sc = float(np.abs(ref).max())
    e_ours = float(np.abs(named[k].grad.double().cpu().numpy() - ref).max())
    e_ref = float(g["g32err/" + k])
    e_orc = float(np.abs(P[k].grad.double().numpy() - ref).max())
    rows.append((e_ours / max(e_ref, e_orc, 1e-4 * sc), k, sc, e_ours, e_ref, e_orc))
rows.sort(reverse=True)
r = np.array([x[0] for x in rows])
print(f"ratio ours/max(ref32,orc32): median {np.median(r):.2f} p90 {np.quantile(r, 0.9):.2f} max {r.max():.2f}")
o = np.array([x[5] / max(x[4], 1e-4 * x[2]) for x in rows])
print(f"ratio orc32/ref32: median {np.median(o):.2f} p90 {np.quantile(o, 0.9):.2f} max {o.max():.2f}")
for x in rows[:25]:
    print(f"{x[0]:7.2f} {x[1]:55s} scale {x[2]:10.4g} ours {x[3]:9.3g} ref32 {x[4]:9.3g} orc32 {x[5]:9.3g}")
