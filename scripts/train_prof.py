"""One B=32 3DPW training step (bench.train_leg's eager step) run `steps`
times, for rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
from engine import mpjpe_error_3d  # noqa: E402
from model import get_model  # noqa: E402


def main(B=32, steps=10):
    dev = torch.device("cuda", 0)
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    torch.manual_seed(0)
    m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
    m._dstd_inplace_grads = True
    opt = torch.optim.Adam(m.parameters(), lr=3e-3, fused=True)  # as bench.train_leg
    g = torch.Generator().manual_seed(1234)
    seq = torch.randn(B, 40, 69, generator=g)
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]
    inv = seq.flip(1).clone()
    inv[:, 10:] = inv[:, 9:10]
    seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
    seq_inv = seq.flip(1).contiguous()
    for _ in range(steps):
        out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
        loss = (mpjpe_error_3d(out.reshape(B, 40, 69), seq) + mpjpe_error_3d(out_i.reshape(B, 40, 69), seq_inv)) / 2
        opt.zero_grad()
        loss.backward()
        opt.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32, int(sys.argv[2]) if len(sys.argv) > 2 else 10)
