#!/usr/bin/env python
"""Interleaved A/B of forward schedule flags within one library: the model's
own eval forward (_forward_native, constants reused) timed per flag set.

  python scripts/flag_ab.py [--config h36m] [--rounds 5] [--steps 50] [--batch 256] name=flags ...
e.g. default=0 whole=32 (include/dstd_gcn.h DSTD_FWD_*)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", default="h36m")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    var = [(v.split("=")[0], int(v.split("=")[1])) for v in a.variants]
    models = {}
    for name, _ in var:  # one model (and workspace cache entry) per variant: each reuses its own constants
        models[name] = bench.load_model(a.config, dev)[0]
    _, opts, _ = bench.load_model(a.config, "cpu")
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(a.batch, T, opts["joints_to_consider"], opts["input_time_frame"], 1).to(dev)
    y = torch.empty_like(x)
    res = {n: [] for n, _ in var}
    with torch.no_grad():
        for _ in range(a.rounds):
            for name, fl in var:
                m = models[name]
                for _ in range(3):
                    m._forward_native(x, y, arith=fl)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    m._forward_native(x, y, arith=fl)
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for name, _ in var:
        r = res[name]
        print(f"{a.config} B={a.batch} {name}: median {np.median(r):.4f} ms (min {min(r):.4f}, max {max(r):.4f})")


if __name__ == "__main__":
    main()
