"""A module on a second GPU called while another device is current
(include/dstd_gcn.h: every entry point launches on the device of its stream,
or of its first device pointer when the stream is the null stream --
csrc/dstd_common.h StreamDeviceGuard).  Skipped on one-GPU boxes."""
import copy

import numpy as np
import pytest
import torch

from conftest import group, load_npz
from model import get_model

pytestmark = pytest.mark.gpu

needs2 = pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                            reason="needs two GPUs")


def _h36m():
    d = load_npz("model_h36m.npz")
    opts = {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "sd/").items()})
    return m.eval(), torch.from_numpy(d["x"].copy())


@needs2
def test_eval_forward_on_second_device_while_first_is_current():
    m, x = _h36m()
    m0, m1 = copy.deepcopy(m).to("cuda:0"), m.to("cuda:1")
    torch.cuda.set_device(0)
    with torch.no_grad():
        y0 = m0(x.to("cuda:0"))
        y1 = m1(x.to("cuda:1"))  # null stream of cuda:1; cuda:0 current
    torch.cuda.synchronize(0)
    torch.cuda.synchronize(1)
    assert y1.device == torch.device("cuda:1")
    assert torch.equal(y0.cpu(), y1.cpu())


@needs2
def test_train_step_on_second_device_while_first_is_current():
    from engine import mpjpe_error_3d
    m, x = _h36m()
    m.train()
    m0, m1 = copy.deepcopy(m).to("cuda:0"), m.to("cuda:1")
    torch.cuda.set_device(0)
    tg = torch.randn(x.shape[0], x.shape[1], x.shape[2] * x.shape[3], generator=torch.Generator().manual_seed(3))
    grads = []
    for mm, dev in ((m0, "cuda:0"), (m1, "cuda:1")):
        loss = mpjpe_error_3d(mm(x.to(dev)).reshape(tg.shape), tg.to(dev))
        loss.backward()
        grads.append([p.grad.detach().cpu().numpy() for p in mm.parameters() if p.grad is not None])
    assert len(grads[0]) == len(grads[1]) > 0
    for a, b in zip(*grads):
        np.testing.assert_array_equal(a, b)
