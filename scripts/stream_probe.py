#!/usr/bin/env python
"""Probe: the eval forward with the batch split into S chunks, each chunk's
whole forward on its own HIP stream (own workspace), so one chunk's
adjacency launches can overlap another chunk's GC launches.  Prints ms/step
per S and checks every S gives the S=1 output bit for bit."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model(os.environ.get("CFG", "h36m"), dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    B = int(os.environ.get("B", "256"))
    x = bench.synth_input(B, T, V, opts["input_time_frame"], 1234).to(dev)
    lanes = [int(s) for s in os.environ.get("LANES", "1,2,3,4").split(",")]
    streams = [torch.cuda.Stream(dev) for _ in range(max(lanes))]
    main_s = torch.cuda.current_stream(dev)
    ref = None

    def fwd(S, y):
        if S == 1:
            model._forward_native(x, y)
            return
        for s in streams[:S]:
            s.wait_stream(main_s)
        for s, xc, yc in zip(streams[:S], x.chunk(S), y.chunk(S)):
            with torch.cuda.stream(s):
                model._forward_native(xc, yc)
        for s in streams[:S]:
            main_s.wait_stream(s)

    res = {S: [] for S in lanes}
    with torch.no_grad():
        for rep in range(3):
            for S in lanes:
                y = torch.empty_like(x)
                for _ in range(10):
                    fwd(S, y)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(100):
                    fwd(S, y)
                torch.cuda.synchronize()
                res[S].append((time.perf_counter() - t0) * 10)
                if ref is None:
                    ref = y.clone()
                elif not torch.equal(ref, y):
                    print(f"S={S}: output differs, max {float((ref - y).abs().max()):.3e}")
    for S in lanes:
        ms = min(res[S])
        print(f"S={S}: {ms:.4f} ms/step  {B / ms * 1e3:,.0f} seq/s  (reps {['%.4f' % v for v in res[S]]})")


if __name__ == "__main__":
    main()
