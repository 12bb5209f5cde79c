"""Bisection of the DSTD_TF_HOISTW build of k_temporal_fused:
workgroup 0's LDS planes (H36M fixture block) from two -DDSTD_TF_DUMPP builds,
compared half by half: which joints / planes / frames / slots differ."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import dstd_native as native
from conftest import group, load_npz
from model import DSTDGCB
d = load_npz("dstdgcb.npz")
name = "b_64_64_h36m"
T, V, SL = 35, 22, 40
PJ = 2 * T * SL + 8
dumps = {}
for lib in sys.argv[1:]:
    native._lib = None
    native.LIB_PATH = os.path.join(ROOT, "dstd-gcn_amd", lib)
    L = native.lib()
    blk = DSTDGCB(64, 64, T, V, "h36m")
    blk.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, f"{name}/sd/").items()})
    blk = blk.to("cuda:0").eval()
    x = torch.from_numpy(d[f"{name}/x"]).to("cuda:0")
    with torch.no_grad():
        blk(x)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint * (64 * 1024))()
    native.check(L.dstd_debug_planes(buf), "dstd_debug_planes")
    h = np.frombuffer(buf, dtype=np.uint16)[:V * PJ].reshape(V, PJ)
    dumps[lib] = h[:, :2 * T * SL].reshape(V, 2, T, SL)
ref, tst = dumps[sys.argv[1]], dumps[sys.argv[2]]
bad = ref != tst
print("differing halves", int(bad.sum()), "of", bad.size)
print("per joint", bad.sum(axis=(1, 2, 3)).tolist())
print("per plane (hi, lo)", bad.sum(axis=(0, 2, 3)).tolist())
print("per frame q", bad.sum(axis=(0, 1, 3)).tolist())
print("per slot", bad.sum(axis=(0, 1, 2)).tolist())
idx = np.argwhere(bad)[:12]
for j, pl, q, sl in idx:
    print(f"  joint {j} plane {pl} q {q} slot {sl}: {ref[j, pl, q, sl]:#06x} vs {tst[j, pl, q, sl]:#06x}")
