#!/usr/bin/env python
"""Whole-model launch (DSTD_FWD_WHOLE_MODEL, k_model_fused) against the
per-block schedule on the same input: per-sample max |diff|, how many samples
agree bit for bit, on the first call (descriptors uploaded) and the second
(reused).  Diagnostic for the experimental schedule."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import dstd_native as native  # noqa: E402

dev = torch.device("cuda", 0)
for cfg in ("h36m", "cmu"):
    m, opts, _ = bench.load_model(cfg, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    x = bench.synth_input(256, T, V, opts["input_time_frame"], 1).to(dev)
    y0, y1, y2 = (torch.empty_like(x) for _ in range(3))
    with torch.no_grad():
        m._forward_native(x, y0, arith=0)
        m._forward_native(x, y1, arith=native.FWD_WHOLE_MODEL)
        m._forward_native(x, y2, arith=native.FWD_WHOLE_MODEL)
    torch.cuda.synchronize()
    for name, y in (("first", y1), ("reuse", y2)):
        d = (y - y0).abs().reshape(256, -1).amax(1)
        print(cfg, name, "equal samples", int((d == 0).sum()), "of 256; max diff", float(d.max()),
              "first bad", int(torch.nonzero(d)[0]) if (d > 0).any() else -1,
              "finite", bool(torch.isfinite(y).all()), "max|y0|", float(y0.abs().max()))
    # per-frame / per-joint pattern of sample 0's difference
    e = (y1 - y0)[0].abs()
    print(cfg, "sample 0 diff by frame", [round(float(v), 3) for v in e.amax((1, 2))[:T]])
