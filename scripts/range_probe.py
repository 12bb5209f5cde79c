"""Range probe: a freshly constructed H36M model (yaml
options, untouched BN) and mm-scale inputs, split vs fp32 vs the fp64 oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
import numpy as np, torch
from model import get_model
from oracle import dstdgcn_oracle as O

def rel(y, r):
    return float(np.abs(np.asarray(y, np.float64) - r).max() / np.abs(r).max())

torch.manual_seed(0)
opts = dict(input_channels=6, input_time_frame=10, output_time_frame=25, st_gcnn_dropout=0.1,
            joints_to_consider=22, num_feature=64, num_layers=5, layout="h36m")
m = get_model("dstdgcn", dstdgcn=opts)
sd = {k: v.clone() for k, v in m.state_dict().items()}
g = torch.Generator().manual_seed(1)
for scale in (1.0, 1000.0):
    x = torch.randn(4, 35, 22, 3, generator=g) * scale
    x[:, 10:] = x[:, 9:10]
    y64 = O.dstdgcn(x, sd, 5).numpy()
    y32 = O.dstdgcn(x, sd, 5, dtype=torch.float32).numpy()
    mg = m.to("cuda:0").eval()
    out = {}
    for prec in ("split", "fp32"):
        with torch.no_grad():
            out[prec] = mg.set_gc_arithmetic(prec)(x.to("cuda:0")).cpu().numpy()
    print(f"scale {scale}: max|y64| {np.abs(y64).max():.3e} ref32 {rel(y32, y64):.2e} "
          f"split {rel(out['split'], y64):.2e} finite {np.isfinite(out['split']).all()} "
          f"fp32 {rel(out['fp32'], y64):.2e}", flush=True)
