#!/usr/bin/env python
"""Per-phase cycle breakdown of the wave kernels (library built with -DDSTD_STAMPS).

  make -C dstd-gcn_amd VARIANT=stamps DEFS=-DDSTD_STAMPS
  python scripts/stamps.py dstd-gcn_amd/libdstd_gcn_stamps.so [--steps 5]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import dstd_native as native  # noqa: E402

PHASES = {
    0: ["conv0(+x wait)", "adj wait", "agg0", "conv1", "R+x issue", "agg1", "glds+epilogue"],
    1: ["conv(+x wait)", "adj wait", "x issue+agg", "glds issue", "epilogue VALU+st", "PQ mfma", "PQ stores"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    native._lib = None
    os.environ["DSTD_LIB"] = os.path.abspath(a.lib)
    native.LIB_PATH = os.path.abspath(a.lib)
    L = native.lib()
    fn = L.dstd_debug_stamps
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model("h36m", dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    x = bench.synth_input(a.batch, T, V, opts["input_time_frame"], 1).to(dev)
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    with torch.no_grad():
        model(x)
        torch.cuda.synchronize()
        for k in (0, 1):
            fn(k, buf.ctypes.data, buf.size, 1)
        for _ in range(a.steps):
            model(x)
        torch.cuda.synchronize()
    units = {0: a.batch * ((T + 1) // 2) * 5, 1: a.batch * V * 6}  # 64->64 launches per forward
    for k in (0, 1):
        fn(k, buf.ctypes.data, buf.size, 1)
        st = buf.reshape(4096, 8).astype(np.float64)
        tot = st.sum(axis=0) / (units[k] * a.steps)
        name = "spatial" if k == 0 else "temporal"
        print(f"{name}: cycles per unit (s_memtime) total {tot.sum():.0f}")
        for i, p in enumerate(PHASES[k]):
            print(f"   {p:18s} {tot[i]:8.0f}")


if __name__ == "__main__":
    main()
