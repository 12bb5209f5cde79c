"""Print bench.train_leg's B=32 training-step line (eager + graph replay) for
the library / environment this process was started with (A/B of training-path
kernels across runs: e.g. DSTD_TRAIN_AGG_GEMM=1 for the strided-GEMM
aggregation products)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
import bench  # noqa: E402

if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    out = bench.train_leg(torch.device("cuda", 0), B, 20, 5)
    print(tag, json.dumps(out), flush=True)
