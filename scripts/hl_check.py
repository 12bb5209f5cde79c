#!/usr/bin/env python
"""Split-f16 vs exact-fp32 GC arithmetic on the GPU, per block and per model,
for every specialised (T, V): max|split - fp32| / max|fp32|.  A debugging aid
for the dstd_hilo.hip kernels (the parity tests proper are tests/test_gpu_parity.py).

  python scripts/hl_check.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import dstd_native  # noqa: E402
from model import DSTDGCB, get_model  # noqa: E402
from oracle import dstdgcn_oracle as O  # noqa: E402

DEV = "cuda:0"
SHAPES = [("h36m", 10, 25, 22), ("cmu", 10, 25, 25), ("3dpw", 10, 30, 23), ("h36m", 50, 25, 22)]


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def both(fn, ref=None):
    out = {}
    for mode in ("fp32", "split"):
        prev = dstd_native.set_gc_precision(mode)
        with torch.no_grad():
            out[mode] = fn().double().cpu()
        dstd_native.set_gc_precision(prev)
    if ref is None:
        return rel(out["split"], out["fp32"])
    return rel(out["split"], out["fp32"]), rel(out["fp32"], ref), rel(out["split"], ref)


def randomise(m):
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith(("alpha_sm", "alpha_tm")):
                p.fill_(0.5)
            elif name.endswith(("W_s", "R_t")):
                p.copy_(0.1 * torch.randn(p.shape))
            elif p.dim() == 1 and "bn" not in name:
                p.copy_(0.1 * torch.randn(p.shape))
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_var.uniform_(0.5, 2.0)


def main():
    torch.manual_seed(0)
    for layout, tin, tout, V in SHAPES:
        T = tin + tout
        blk = DSTDGCB(64, 64, T, V, layout)
        randomise(blk)
        blk = blk.to(DEV).eval()
        x = torch.randn(4, 64, T, V, device=DEV)
        e_blk = both(lambda: blk(x))
        opts = dict(input_channels=6, input_time_frame=tin, output_time_frame=tout, st_gcnn_dropout=0.0,
                    joints_to_consider=V, num_feature=64, num_layers=5, layout=layout)
        m = get_model("dstdgcn", dstdgcn=opts)
        randomise(m)
        m = m.to(DEV).eval()
        xm = torch.randn(4, T, V, 3, device=DEV)
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        ref = O.dstdgcn(xm.cpu(), sd, 5)
        e = both(lambda: m(xm), torch.as_tensor(ref))
        print(f"{layout:5s} T={T:3d} V={V}: block 64->64 split vs fp32 {e_blk:.2e}   model split vs fp32 {e[0]:.2e}, "
              f"fp32 vs oracle {e[1]:.2e}, split vs oracle {e[2]:.2e}", flush=True)


if __name__ == "__main__":
    main()
