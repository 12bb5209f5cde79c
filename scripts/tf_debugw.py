"""Bisection of the DSTD_TF_HOISTW build of k_temporal_fused:
run one fixture block through libdstd_gcn_debugw.so (-DDSTD_TF_HOISTW=1
-DDSTD_TF_DEBUGW) and compare, per row tile, the W fragments held in
registers across the tile loop with a fresh read of the same LDS words."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import dstd_native as native
from conftest import group, load_npz
from model import DSTDGCB
native.LIB_PATH = os.path.join(ROOT, "dstd-gcn_amd", "libdstd_gcn_debugw.so")
L = native.lib()
d = load_npz("dstdgcb.npz")
name = "b_64_64_h36m"
blk = DSTDGCB(64, 64, 35, 22, "h36m")
blk.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, f"{name}/sd/").items()})
blk = blk.to("cuda:0").eval()
x = torch.from_numpy(d[f"{name}/x"]).to("cuda:0")
with torch.no_grad():
    blk(x)
torch.cuda.synchronize()
buf = (ctypes.c_uint * (2 * 512 * 24))()
native.check(L.dstd_debug_w(buf), "dstd_debug_w")
a = np.frombuffer(buf, dtype=np.uint32).reshape(2, 512, 24)
for rt in range(2):
    held, fresh = a[rt, :, :12], a[rt, :, 12:]
    bad = (held != fresh)
    print(f"row tile {rt}: lanes with a differing word {int(bad.any(1).sum())} of 512; "
          f"per word {bad.sum(0).tolist()}")
    idx = np.argwhere(bad.any(1)).ravel()[:4]
    for i in idx:
        print("  thread", int(i), "held", [hex(v) for v in held[i]], "\n         fresh", [hex(v) for v in fresh[i]])
