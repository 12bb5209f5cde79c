#!/usr/bin/env python
"""Print the HIP path's error against every golden fixture (GPU box).

Usage: python scripts/parity_report.py [out.json]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from conftest import group, load_npz, rel_err  # noqa: E402
from model import DSTDGC, DSTDGCB, get_model  # noqa: E402
import test_gpu_parity as G  # noqa: E402

DEV = "cuda:0"


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def run(rep, suffix, arith):
    d = load_npz("dstdgc_ops.npz")
    for name, (mode, cin, cout, T, V) in G.OPS.items():
        ref, kpt = (T, V) if mode == "spatial" else (V, T)
        op = DSTDGC(cin, cout, ref, kpt, mode=mode)
        op.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, f"{name}/sd/").items()})
        op = op.to(DEV).eval()  # the op API always runs the exact-fp32 kernels
        with torch.no_grad():
            y = op(t(d[f"{name}/x"]), t(d[f"{name}/A"]), t(d[f"{name}/alpha"]))
        rep["op/" + name + suffix] = (rel_err(y.cpu().numpy(), d[f"{name}/y64"]), float(d[f"{name}/ref32_err"]))
    d = load_npz("dstdgcb.npz")
    for name, (cin, cout, layout, T, V) in G.BLOCKS.items():
        blk = DSTDGCB(cin, cout, T, V, layout)
        blk.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, f"{name}/sd/").items()})
        blk = blk.to(DEV).eval()
        blk.gc_arithmetic = arith
        with torch.no_grad():
            y = blk(t(d[f"{name}/x"]))
        rep["block/" + name + suffix] = (rel_err(y.cpu().numpy(), d[f"{name}/y64"]), float(d[f"{name}/ref32_err"]))
    for tag in G.MODELS:
        m, dd, _, _ = G.load_model(tag, arith)
        with torch.no_grad():
            y = m(t(dd["x"]))
        rep["model/" + tag + suffix] = (rel_err(y.cpu().numpy(), dd["y64"]), float(dd["ref32_err"]))


def main():
    """Both GC arithmetics of the library (split-f16 default, exact fp32)."""
    rep = {}
    for arith in ("split", "fp32"):
        run(rep, "/" + arith, arith)
    # the reference forward itself on this GPU in fp32 (torch-ROCm ops: the
    # oracle is an op-for-op restatement of model/dstdgcn.py): its error
    # against the fp64 fixture, beside the CPU fp32 error the fixture holds
    from oracle import dstdgcn_oracle as O
    for tag in G.MODELS:
        _, dd, sd, opts = G.load_model(tag)
        with torch.no_grad():
            y = O.dstdgcn(dd["x"], sd, opts["num_layers"], dtype=torch.float32, device=DEV)
        rep["torch_gpu_fp32/" + tag] = (rel_err(y.cpu().numpy(), dd["y64"]), float(dd["ref32_err"]))
    print(f"{'case':28s} {'hip_err':>10s} {'ref32_err':>10s}  ratio")
    for k, (e, r) in rep.items():
        print(f"{k:28s} {e:10.3e} {r:10.3e}  {e / max(r, 1e-30):6.2f}")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump({k: {"hip_err": e, "ref32_err": r, "ratio": e / max(r, 1e-30)} for k, (e, r) in rep.items()},
                      f, indent=1)


if __name__ == "__main__":
    main()
