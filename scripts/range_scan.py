"""Magnitude scan of one fresh DSTDGCB (homogeneous at init: zero biases,
untouched BN): block(2^k x) = 2^k block(x); split vs fp32 per k, per library."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import dstd_native as native
from model import DSTDGCB
from oracle import dstdgcn_oracle as O
from conftest import rel_err
libs = sys.argv[1:] or [native.LIB_PATH]
torch.manual_seed(3)
blk = DSTDGCB(64, 64, 35, 22, "h36m")
sd = {k: v.clone() for k, v in blk.state_dict().items()}
x = torch.randn(2, 64, 35, 22)
y64 = O.dstdgcb_forward(x, sd).numpy()
blk = blk.to("cuda:0").eval()
for path in libs:
    native._lib = None
    native.LIB_PATH = path
    native.lib()
    row = []
    for k in range(0, 26, 2):
        with torch.no_grad():
            y = blk((x * 2.0 ** k).to("cuda:0")).cpu().numpy() / 2.0 ** k
        row.append(f"{k}:{rel_err(y, y64):.1e}")
    print(os.path.basename(path), " ".join(row), flush=True)
