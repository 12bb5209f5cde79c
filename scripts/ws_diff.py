"""Byte ranges where two library variants leave a different model workspace
after one forward (zero-filled before), e.g. to locate which intermediate
(adjacency planes, P/Q, activations) first differs.

  python scripts/ws_diff.py --config h36m libA.so libB.so   (paths under dstd-gcn_amd/)
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
import bench  # noqa: E402
import dstd_native as native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--config", default="h36m")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model(a.config, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    x = bench.synth_input(a.batch, T, V, opts["input_time_frame"], 1).to(dev)
    ws = {}
    for lib in a.libs:
        native._lib = None
        native.LIB_PATH = os.path.join(ROOT, "dstd-gcn_amd", lib)
        model._native = None
        native._ws_cache.clear()
        L = native.lib()
        nbytes = L.dstd_model_workspace_bytes(a.batch, T, V, model.num_feature, model.num_layers)
        native.workspace(dev, nbytes).zero_()
        with torch.no_grad():
            model(x)
        torch.cuda.synchronize()
        buf = next(iter(native._ws_cache.values()))[0]
        ws[lib] = buf[:nbytes].cpu().numpy().view(np.uint16)
    d = np.nonzero(ws[a.libs[0]] != ws[a.libs[1]])[0]
    print(f"{a.config} B={a.batch}: {len(d)} of {len(ws[a.libs[0]])} halves differ")
    if len(d):
        cuts = np.nonzero(np.diff(d) > 4096)[0]
        starts = np.r_[d[0], d[cuts + 1]]
        ends = np.r_[d[cuts], d[-1]]
        for s, e in zip(starts, ends):
            n = int(((d >= s) & (d <= e)).sum())
            print(f"  bytes [{2 * s:#x}, {2 * e + 2:#x}) {n} halves differ")


if __name__ == "__main__":
    main()
