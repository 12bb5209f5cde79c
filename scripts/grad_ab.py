"""Gradients of one B=32 3DPW training step (bench.train_leg's step without
the optimizer) for the library this process was started with (DSTD_LIB),
saved to an .npz; with --compare, the largest relative difference per
parameter between two such files (A/B of training-path kernel variants:
identical sums print 0).

  DSTD_LIB=.../libdstd_gcn_x.so python scripts/grad_ab.py out_x.npz
  python scripts/grad_ab.py --compare out_a.npz out_b.npz
"""
import os
import sys

import numpy as np


def dump(path, B=32):
    import torch
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "dstd-gcn_amd")]
    from engine import mpjpe_error_3d
    from model import get_model
    dev = torch.device("cuda", 0)
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    torch.manual_seed(0)
    m = get_model("dstdgcn", dstdgcn=opts).to(dev).train()
    m._dstd_inplace_grads = True
    g = torch.Generator().manual_seed(1234)
    seq = torch.randn(B, 40, 69, generator=g)
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]
    inv = seq.flip(1).clone()
    inv[:, 10:] = inv[:, 9:10]
    seq, inp, inv = seq.to(dev), inp.to(dev), inv.to(dev)
    out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
    loss = (mpjpe_error_3d(out.reshape(B, 40, 69), seq) + mpjpe_error_3d(out_i.reshape(B, 40, 69), seq.flip(1))) / 2
    loss.backward()
    torch.cuda.synchronize()
    np.savez(path, **{n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters() if p.grad is not None})
    print("saved", path, "loss", float(loss.detach()))


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    rel, nid = {}, 0
    for k in A.files:
        x, y = A[k].astype(np.float64), Bz[k].astype(np.float64)
        rel[k] = float(np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-30))  # (norm-relative: near-zero
        nid += int(np.array_equal(A[k], Bz[k]))                                #  noise tensors do not dominate)
    w = sorted(rel, key=rel.get)[-3:]
    print(f"{os.path.basename(b)} vs {os.path.basename(a)}: {nid}/{len(A.files)} tensors identical, "
          f"median |d|/|g| {np.median(list(rel.values())):.2e}, worst " + ", ".join(f"{k} {rel[k]:.2e}" for k in w))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
