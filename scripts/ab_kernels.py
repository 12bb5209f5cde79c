#!/usr/bin/env python
"""A/B per-kernel-family times of library variants, interleaved in one process.

  python scripts/ab_kernels.py lib1.so lib2.so ... [--rounds 5 --steps 10 --batch 256 --config h36m]
Each library is loaded in turn (ctypes, separate handles) and timed with the
dstd_model_fwd_profiled event brackets; rounds interleave the variants.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import dstd_native as native  # noqa: E402


def load(path):
    native._lib = None
    os.environ["DSTD_LIB"] = path
    native.LIB_PATH = path
    return native.lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--config", default="h36m")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model(a.config, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(a.batch, T, opts["joints_to_consider"], opts["input_time_frame"], 1).to(dev)
    y = torch.empty_like(x)
    libs = {p: load(p) for p in a.libs}
    res = {p: {} for p in a.libs}
    with torch.no_grad():
        for r in range(a.rounds):
            for p, L in libs.items():
                native._lib = L
                model._native = None
                for _ in range(2):
                    model(x)
                prof = bench.Profiler(L, a.steps * 40, 0x7F)
                for _ in range(a.steps):
                    bench.forward_profiled(model, x, y, prof)
                torch.cuda.synchronize()
                per = {}
                for k, _, ms in prof.elapsed():
                    per[native.KIND_NAMES[k]] = per.get(native.KIND_NAMES[k], 0.0) + ms / a.steps
                prof.close()
                for k, v in per.items():
                    res[p].setdefault(k, []).append(v)
                # wall clock of unbracketed forwards (kernel-boundary costs included)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5 * a.steps):
                    model._forward_native(x, y)
                torch.cuda.synchronize()
                res[p].setdefault("wall", []).append((time.perf_counter() - t0) * 1e3 / (5 * a.steps))
    for p in a.libs:
        tot = sum(np.median(v) for k, v in res[p].items() if k != "wall")
        print(os.path.basename(p), f"wall {np.median(res[p]['wall']):.4f} (min {min(res[p]['wall']):.4f}) "
              f"kernels {tot:.4f} ms/step",
              {k: round(float(np.median(v)), 4) for k, v in res[p].items() if k != "wall"})


if __name__ == "__main__":
    main()
