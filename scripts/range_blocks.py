"""Per-block split-vs-oracle errors on the fresh (untouched-BN) H36M model:
feeds every DSTDGCB the fp64 oracle's own input to that block."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import test_gpu_parity as G
from oracle import dstdgcn_oracle as O
from conftest import rel_err

m = G.fresh_h36m(9)
sd = {k: v.clone().double() for k, v in m.state_dict().items() if not k.endswith("num_batches_tracked")}
x = G.synth(4, 35, 22, 10, 44).double()
residual = x[:, -1:]
h = torch.cat((x, x - residual), dim=-1).permute(0, 3, 1, 2)
blocks = [("conv_st_in", m.conv_st_in.stgcn[0][0], "conv_st_in.stgcn.0.0.")]
blocks += [(f"enc{i}", m.encoders[i][0].stgcn[0][0], f"encoders.{i}.0.stgcn.0.0.") for i in range(5)]
blocks += [("conv_st_out", m.conv_st_out.stgcn[0][0], "conv_st_out.stgcn.0.0.")]
m = m.to("cuda:0").eval()
for bi, (name, blk, pre) in enumerate(blocks):
    y64 = O.dstdgcb(h, O.sub(sd, pre))
    res = {}
    for prec in ("split", "fp32"):
        blk.gc_arithmetic = prec
        with torch.no_grad():
            res[prec] = blk(h.float().to("cuda:0")).cpu().numpy()
    print(f"{name:12s} max|x| {h.abs().max():.3e} max|y| {y64.abs().max():.3e} split {rel_err(res['split'], y64.numpy()):.2e} "
          f"fp32 {rel_err(res['fp32'], y64.numpy()):.2e}", flush=True)
    if bi == 0:
        h = O.prelu(O.batchnorm(y64, O.sub(sd, "bn_in.bn.")), sd["prelu.weight"])
    elif bi < 6:
        e = f"encoders.{bi - 1}."
        h = O.prelu(O.batchnorm(y64 + h, O.sub(sd, e + "1.bn.")), sd[e + "2.weight"])
