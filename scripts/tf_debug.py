"""Fused vs unfused temporal path on one DSTDGCB (fixture b_64_64_h36m):
max |diff| per joint and per frame (which part of the planes is wrong)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import dstd_native as native
from conftest import group, load_npz
from model import DSTDGCB
d = load_npz("dstdgcb.npz")
name = sys.argv[1] if len(sys.argv) > 1 else "b_64_64_h36m"
layout = name.rsplit("_", 1)[1]
V = {"h36m": 22, "cmu": 25, "3dpw": 23}[layout]
blk = DSTDGCB(64, 64, 35, V, layout)
blk.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, f"{name}/sd/").items()})
blk = blk.to("cuda:0").eval()
x = torch.from_numpy(d[f"{name}/x"]).to("cuda:0")
out = {}
libs = ["libdstd_gcn_nofused.so"] + (sys.argv[2:] or ["libdstd_gcn.so"])
for lib in libs:
    native._lib = None
    native.LIB_PATH = os.path.join(ROOT, "dstd-gcn_amd", lib)
    with torch.no_grad():
        out[lib] = blk(x).double().cpu().numpy()  # [B, C, T, V]
ref = np.abs(out["libdstd_gcn_nofused.so"]).max()
for lib in libs[1:]:
    diff = np.abs(out[lib] - out["libdstd_gcn_nofused.so"])
    print(lib, "rel", diff.max() / ref)
    print("  per joint", np.round(diff.max(axis=(0, 1, 2)) / ref, 3).tolist())
    print("  per frame", np.round(diff.max(axis=(0, 1, 3)) / ref, 3).tolist())
