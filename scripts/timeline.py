#!/usr/bin/env python
"""Workgroup timeline of the adjacency kernels (library built with -DDSTD_STAMPS).

  python scripts/timeline.py dstd-gcn_amd/libdstd_gcn_stamps.so [--hl]
(--hl: the split-f16 adjacency kernels of dstd_hilo.hip).  Runs one forward, then reads the last launch's per-workgroup s_memrealtime
stamps (entry, staging done, compute done, exit; 100 MHz) for each mode.
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
    native._lib = None
    os.environ["DSTD_LIB"] = lib
    native.LIB_PATH = lib
    L = native.lib()
    fn = L.dstd_debug_timeline_hl if "--hl" in sys.argv else L.dstd_debug_timeline
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model("h36m", dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(256, T, opts["joints_to_consider"], opts["input_time_frame"], 1).to(dev)
    with torch.no_grad():
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
    buf = np.zeros(2048 * 4, dtype=np.uint64)
    names = {0: "k_adj_hl<0>", 1: "k_adj_hl<1>", 2: "k_temporal_fused phase 3 (start, E/F, tiles, drained)",
             3: "k_temporal_fused C=64 (entry, chunk-0 phase 1, units, exit)",
             4: "k_temporal_fused C=64 chunk 0 (entry, phase-1 prologue, wave 0's tiles, stage)"}
    for mode in ((0, 1, 2, 3, 4) if "--hl" in sys.argv else (0, 1)):
        fn(mode, buf.ctypes.data, buf.size)
        raw = buf.reshape(2048, 4).copy()
        raw = raw[raw[:, 0] > 0]
        hw = None
        if not len(raw):
            print(f"mode {mode} ({names.get(mode)}): no stamps")
            continue
        if "--hl" in sys.argv and mode < 2:  # slot 3 holds (XCC_ID << 32) | HW_ID: placement per workgroup
            hw = raw[:, 3].copy()
            raw[:, 3] = raw[:, 2]
        tl = raw.astype(np.float64)
        t0 = tl[:, 0].min()
        us = (tl - t0) / 100.0  # 100 MHz -> us
        print(f"mode {mode} ({names.get(mode)}): {len(tl)} workgroups, span {us[:, 3].max():.2f} us")
        for name, col in (("entry", 0), ("staged", 1), ("computed", 2), ("exit", 3)):
            c = us[:, col]
            print(f"   {name:9s} min {c.min():6.2f}  p50 {np.median(c):6.2f}  p90 {np.percentile(c, 90):6.2f}  max {c.max():6.2f}")
        d = us[:, 2] - us[:, 1]
        print(f"   compute   p50 {np.median(d):6.2f} us; staging p50 {np.median(us[:, 1] - us[:, 0]):6.2f} us")
        if hw is not None:
            hwid = (hw & 0xffffffff).astype(np.int64)
            xcc = (hw >> 32).astype(np.int64) & 0xf
            cu = (hwid >> 8) & 0xf
            sh = (hwid >> 12) & 0x1
            se = (hwid >> 13) & 0x7
            key = xcc * 1000 + se * 100 + sh * 16 + cu
            uniq, cnt = np.unique(key, return_counts=True)
            print(f"   placement: {len(uniq)} distinct CUs, workgroups per CU histogram "
                  f"{dict(zip(*np.unique(cnt, return_counts=True)))}")
            per = {k: c for k, c in zip(uniq, cnt)}
            shared = np.array([per[k] for k in key])
            for x in sorted(set(xcc)):
                sel = xcc == x
                print(f"     XCC {x}: {sel.sum()} WGs, compute p50 {np.median(d[sel]):6.2f} p90 {np.percentile(d[sel], 90):6.2f}"
                      f" max {d[sel].max():6.2f}, staged p50 {np.median(us[sel, 1]):6.2f}")
            for c in sorted(set(shared)):
                sel = shared == c
                print(f"     {c} WG/CU: {sel.sum()} WGs, compute p50 {np.median(d[sel]):6.2f} us, max {d[sel].max():6.2f}")


if __name__ == "__main__":
    main()
