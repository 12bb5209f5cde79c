"""Whole-model forward of library variants on the same input: max |diff| over
max |y| against the first library, and whether the outputs are bit-identical.

  python scripts/model_ab.py --config h36m lib_ref.so lib2.so ...   (paths under dstd-gcn_amd/)
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
import bench  # noqa: E402
import dstd_native as native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="h36m")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, opts, _ = bench.load_model(a.config, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(a.batch, T, opts["joints_to_consider"], opts["input_time_frame"], 1).to(dev)
    out = {}
    for lib in a.libs:
        native._lib = None
        native.LIB_PATH = os.path.join(ROOT, "dstd-gcn_amd", lib)
        model._native = None
        with torch.no_grad():
            out[lib] = model(x).double().cpu()
    ref = out[a.libs[0]]
    for lib in a.libs[1:]:
        d = (out[lib] - ref).abs()
        print(f"{a.config} {lib} vs {a.libs[0]}: rel {float(d.max() / ref.abs().max()):.3e} "
              f"identical {bool(torch.equal(out[lib], ref))} finite {bool(torch.isfinite(out[lib]).all())}")


if __name__ == "__main__":
    main()
