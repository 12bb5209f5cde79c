#!/usr/bin/env python
"""Emulated error of the split-f16 MFMA arithmetic (dstd-gcn_amd/csrc/dstd_hilo.h)
on the reference fixtures.  Every contraction of the CPU oracle runs with its
operands carried as f16 hi/lo pairs (weights power-of-two prescaled, activations
unscaled) and three products (hi*hi + hi*lo + lo*hi); the result is compared with
the reference's fp64 output next to the reference's own fp32 error.

CPU only (test infrastructure, imports the oracle):  python scripts/split_precision.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import dstdgcn_oracle as O  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
_einsum = torch.einsum
WEIGHT_FIRST = ("oc,nctv->notv", "tk,nkvw->ntvw", "vk,nktu->nvtu")  # conv weights are operand 0
MODE = None


def hilo(a, scaled):
    a = a.double()
    s = 1.0
    if scaled:  # power-of-two prescale: max|a| * s < 2^14
        s = 2.0 ** (14 - int(np.frexp(float(a.abs().max()) + 1e-30)[1]))
        a = a * s
    h = a.half().double()
    lo = (a - h).half().double()
    return h / s, lo / s


def einsum(eq, a, b):
    if MODE is None:
        return _einsum(eq, a, b)
    ah, al = hilo(a, eq in WEIGHT_FIRST)
    bh, bl = hilo(b, False)
    out = _einsum(eq, ah, bh) + _einsum(eq, ah, bl) + _einsum(eq, al, bh)
    return out.float().to(a.dtype)


def main():
    global MODE
    shim = type(sys)("torch_shim")
    shim.__dict__.update(torch.__dict__)
    shim.einsum = einsum
    O.torch = shim
    d = np.load(os.path.join(GOLDEN, "dstdgc_ops.npz"))
    for c in sorted({k.split("/")[0] for k in d.files}):
        sd = {k[len(c) + 4:]: torch.from_numpy(d[k]).float() for k in d.files if k.startswith(c + "/sd/")}
        x = torch.from_numpy(d[c + "/x"]).float()
        A = torch.from_numpy(d[c + "/A"]).float()
        al = torch.from_numpy(d[c + "/alpha"]).float()
        mode = "spatial" if c.startswith("s") else "temporal"
        ref = d[c + "/y64"]
        errs = []
        for m in (None, "split"):
            MODE = m
            y = O.dstdgc(x, sd, A, al[0], mode).double().numpy()
            errs.append(np.abs(y - ref).max() / np.abs(ref).max())
        MODE = None
        print(f"{c:18s} ref32 {float(d[c + '/ref32_err']):.2e}  fp32 {errs[0]:.2e}  split {errs[1]:.2e}")
    for fx in ["model_h36m", "model_cmu", "model_3dpw", "model_h36m75"]:
        d2 = np.load(os.path.join(GOLDEN, f"{fx}.npz"))
        opts = {k[4:]: d2[k].item() for k in d2.files if k.startswith("opt/")}
        sd = {k[3:]: d2[k] for k in d2.files if k.startswith("sd/")}
        x = torch.from_numpy(d2["x"])
        ref = O.dstdgcn(x, sd, opts["num_layers"]).numpy()
        MODE = "split"
        y = O.dstdgcn(x, sd, opts["num_layers"], dtype=torch.float32).double().numpy()
        MODE = None
        err = np.abs(y - ref).max() / np.abs(ref).max()
        print(f"{fx:18s} ref32 {float(d2['ref32_err']):.2e}  split {err:.2e}")


if __name__ == "__main__":
    main()
