"""Pin the CPU oracle against fixtures produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import group, load_npz, rel_err
from oracle import dstdgcn_oracle as O

OPS = ["s_64_64_h36m", "s_6_64_h36m", "s_64_3_h36m", "s_64_64_cmu",
       "t_64_64_h36m", "t_3_3_h36m", "t_64_64_3dpw", "t_64_64_h36m75"]
BLOCKS = ["b_64_64_h36m", "b_6_64_h36m", "b_64_3_h36m", "b_64_64_cmu"]
MODELS = ["h36m", "cmu", "3dpw", "h36m75"]


@pytest.mark.parametrize("name", OPS)
def test_oracle_dstdgc_op(name):
    d = load_npz("dstdgc_ops.npz")
    sd = group(d, f"{name}/sd/")
    mode = "spatial" if name.startswith("s_") else "temporal"
    y = O.dstdgc_forward(d[f"{name}/x"], sd, d[f"{name}/A"], d[f"{name}/alpha"], mode)
    assert rel_err(y.numpy(), d[f"{name}/y64"]) < 1e-6


@pytest.mark.parametrize("name", BLOCKS)
def test_oracle_dstdgcb(name):
    d = load_npz("dstdgcb.npz")
    y = O.dstdgcb_forward(d[f"{name}/x"], group(d, f"{name}/sd/"))
    assert rel_err(y.numpy(), d[f"{name}/y64"]) < 1e-6


@pytest.mark.parametrize("tag", MODELS)
def test_oracle_dstdgcn(tag):
    d = load_npz(f"model_{tag}.npz")
    sd = group(d, "sd/")
    y = O.dstdgcn(d["x"], sd, int(d["opt/num_layers"]))
    assert rel_err(y.numpy(), d["y64"]) < 1e-6
    # fp32 restatement lands within the reference's own fp32 error band
    y32 = O.dstdgcn(d["x"], sd, int(d["opt/num_layers"]), dtype=torch.float32)
    assert rel_err(y32.numpy(), d["y64"]) < max(1e-4, 4 * float(d["ref32_err"]))


def test_oracle_mpjpe():
    d = load_npz("engine.npz")
    v = O.mpjpe_error_3d(torch.from_numpy(d["mpjpe/pred"]).double(), torch.from_numpy(d["mpjpe/targ"]).double())
    assert abs(float(v) - float(d["mpjpe/value"])) < 1e-5
