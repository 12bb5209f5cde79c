#!/usr/bin/env python
"""Debug aid: the 64->3 DSTDGCB (conv_st_out) under both GC arithmetics with
the temporal DSTDGC made an identity (conv_f = I, alpha_tm = 0, A_t + R_t = I),
so the block output is the spatial GC output h; then with the real temporal
weights.  Prints max rel differences vs the fp64 oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import dstd_native  # noqa: E402
from model import DSTDGCB  # noqa: E402
from oracle import dstdgcn_oracle as O  # noqa: E402

DEV = "cuda:0"
d = np.load(os.path.join(ROOT, "tests", "golden", "dstdgcb.npz"))
name = sys.argv[1] if len(sys.argv) > 1 else "b_64_3_h36m"
cin, cout = (64, 3) if "64_3" in name else (6, 64) if "6_64" in name else (64, 64)
sd = {k[len(name) + 4:]: torch.from_numpy(d[k]) for k in d.files if k.startswith(name + "/sd/")}
x = torch.from_numpy(d[name + "/x"])
for ident in (True, False):
    s2 = {k: v.clone() for k, v in sd.items()}
    if ident:
        s2["conv_t.0.conv_f.weight"] = torch.eye(cout).reshape(cout, cout, 1, 1)
        s2["conv_t.0.conv_f.bias"].zero_()
        s2["alpha_tm"].zero_()
        s2["A_t"] = torch.eye(35).reshape(1, 35, 35)
        s2["R_t"] = torch.zeros(1, 35, 35)
    ref = O.dstdgcb_forward(x, s2).numpy() if hasattr(O, "dstdgcb_forward") else None
    out = {}
    for mode in ("fp32", "split"):
        blk = DSTDGCB(cin, cout, 35, 22, "h36m")
        blk.load_state_dict(s2)
        blk = blk.to(DEV).eval()
        prev = dstd_native.set_gc_precision(mode)
        with torch.no_grad():
            out[mode] = blk(x.to(DEV)).double().cpu().numpy()
        dstd_native.set_gc_precision(prev)
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    print(f"{name} identity-temporal={ident}: split vs fp32 {rel(out['split'], out['fp32']):.3e}",
          f"fp32 vs oracle {rel(out['fp32'], ref):.3e} split vs oracle {rel(out['split'], ref):.3e}" if ref is not None else "")
    if ident:
        diff = np.abs(out["split"] - out["fp32"]).max(axis=(0, 2))  # per channel, joint
        print("   max |diff| per (channel, joint):", np.round(diff, 4).tolist())
