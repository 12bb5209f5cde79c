"""Whole-model error ratio distribution (err / ref32 on the same input) over
many synthetic inputs: split path, exact-fp32 path, and the reference forward
in fp32 on this GPU (torch-ROCm), per fixture model.  ref32 = the fp32 CPU
oracle's error (the reference's own fp32 error on that input)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import test_gpu_parity as G
from oracle import dstdgcn_oracle as O
from conftest import rel_err
N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
for tag in sys.argv[2:] or G.MODELS:
    m, d, sd, opts = G.load_model(tag)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    rat = {"split": [], "fp32": [], "torch_gpu": []}
    for i in range(N):
        x = G.synth(4, T, V, opts["input_time_frame"], 1000 + i)
        y64 = O.dstdgcn(x, sd, opts["num_layers"]).numpy()
        r32 = rel_err(O.dstdgcn(x, sd, opts["num_layers"], dtype=torch.float32).numpy(), y64)
        for prec in ("split", "fp32"):
            with torch.no_grad():
                y = m.set_gc_arithmetic(prec)(x.to(G.DEV)).cpu().numpy()
            rat[prec].append(rel_err(y, y64) / r32)
        with torch.no_grad():
            yt = O.dstdgcn(x, sd, opts["num_layers"], dtype=torch.float32, device=G.DEV).cpu().numpy()
        rat["torch_gpu"].append(rel_err(yt, y64) / r32)
    print(tag, {k: f"median {np.median(v):.2f} p90 {np.percentile(v, 90):.2f} max {max(v):.2f}" for k, v in rat.items()},
          flush=True)
