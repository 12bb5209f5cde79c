#!/usr/bin/env python
"""Phase timeline of the per-sample block kernel (k_block_fused, library built
with -DDSTD_STAMPS): one H36M B=256 forward, then per workgroup of the last
64 -> 64 block launch the spatial GC (entry -> units done), the barrier, the
fused temporal body's phase 1 (temporal adjacency in LDS), phase 2 (joint
units) and phase 3 (next block's spatial planes), from the s_memrealtime
stamps of modes 5 and 3 (one clock, 100 MHz).

  python scripts/bf_timeline.py dstd-gcn_amd/libdstd_gcn_stamps.so [--config h36m]
"""
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


def main():
    lib = os.path.abspath(sys.argv[1])
    cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "h36m"
    native._lib = None
    os.environ["DSTD_LIB"] = lib
    native.LIB_PATH = lib
    L = native.lib()
    fn = L.dstd_debug_timeline_hl
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model(cfg, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(256, T, opts["joints_to_consider"], opts["input_time_frame"], 1).to(dev)
    with torch.no_grad():
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
    st = {}
    for mode in (5, 3, 2):
        buf = np.zeros(2048 * 4, dtype=np.uint64)
        fn(mode, buf.ctypes.data, buf.size)
        st[mode] = buf.reshape(2048, 4)[:256].astype(np.float64)
    m5, m3, m2 = st[5], st[3], st[2]
    ok = (m5[:, 0] > 0) & (m3[:, 0] > 0)
    t0 = m5[ok, 0].min()
    us = lambda a: (a[ok] - t0) / 100.0  # noqa: E731
    e5, e3, e2 = us(m5), us(m3), us(m2)
    phases = [("spatial GC (entry -> units done)", e5[:, 1] - e5[:, 0]),
              ("barrier", e5[:, 2] - e5[:, 1]),
              ("temporal phase 1 (prologue + tiles + barrier)", e3[:, 1] - e3[:, 0]),
              ("temporal phase 2 (stage + joint units)", e3[:, 2] - e3[:, 1]),
              ("phase 3 (next block's spatial planes)", e3[:, 3] - e3[:, 2]),
              ("phase 3 prologue (E/F ready)", e2[:, 1] - e2[:, 0]),
              ("phase 3 wave 0: tiles issued", e2[:, 2] - e2[:, 1]),
              ("phase 3 wave 0: its stores drained", e2[:, 3] - e2[:, 2]),
              ("phase 3 wave 0 done -> workgroup exit", e5[:, 3] - e2[:, 3]),
              ("workgroup total", e5[:, 3] - e5[:, 0])]
    print(f"{cfg}: {ok.sum()} workgroups, launch span {e5[:, 3].max():.2f} us, entries {e5[:, 0].min():.2f}.."
          f"{e5[:, 0].max():.2f} us, exits {e5[:, 3].min():.2f}..{e5[:, 3].max():.2f} us")
    for name, d in phases:
        print(f"  {name:48s} p10 {np.percentile(d, 10):6.2f}  p50 {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}"
              f"  max {d.max():6.2f} us")


if __name__ == "__main__":
    main()
