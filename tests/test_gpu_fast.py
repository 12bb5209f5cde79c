"""MI355X parity of the channels-last variant (model/dstdgcn_fast.py, SURVEY
§8(f) row 4) against the reference's own outputs (dstdgcn_fast.npz, made by
running reference dstdgcn_fast.py) and the CPU oracle's fast_* restatement.
Bars as test_gpu_parity.py: 1e-4 per op / block, conftest.model_tol for
whole models; gradients as test_gpu_train.py (error over the fp32 noise of
two other implementations)."""
import copy

import numpy as np
import pytest
import torch

from conftest import group, load_npz, model_tol, rel_err
from model import dstdgcn_fast as F
from model.dstdgcn import invalidate_native_cache
from oracle import dstdgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

OPS = {"op_s_64_64": ("spatial", 64, 64, 35, 22), "op_s_6_64": ("spatial", 6, 64, 35, 22),
       "op_t_64_64": ("temporal", 64, 64, 35, 22), "op_t_64_64_3dpw": ("temporal", 64, 64, 40, 23)}
BLOCKS = {"blk_64_64": (64, 64, "h36m", 35, 22), "blk_6_64": (6, 64, "h36m", 35, 22),
          "blk_64_3": (64, 3, "h36m", 35, 22), "blk_64_64_cmu": (64, 64, "cmu", 35, 25)}


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _load(mod, sd):
    mod.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return mod


def _model(tag, d):
    p = f"model_{tag}/"
    opts = {k[len(p + "opt/"):]: d[k].item() for k in d.files if k.startswith(p + "opt/")}
    return _load(F.DSTDGCN(**opts), group(d, p + "sd/")).to(DEV).eval(), opts


@pytest.mark.parametrize("name", list(OPS))
def test_fast_dstdgc_op(name):
    d = load_npz("dstdgcn_fast.npz")
    mode, cin, cout, T, V = OPS[name]
    ref, kpt = (T, V) if mode == "spatial" else (V, T)
    op = _load(F.DSTDGC(cin, cout, ref, kpt, mode=mode), group(d, f"{name}/sd/")).to(DEV).eval()
    with torch.no_grad():
        y = op(t(d[f"{name}/x"]), t(d[f"{name}/A"]), t(d[f"{name}/alpha"]))
    assert y.shape == (1, T, V, cout)
    assert rel_err(y.cpu().numpy(), d[f"{name}/y64"]) <= 1e-4


@pytest.mark.parametrize("name", list(BLOCKS))
@pytest.mark.parametrize("arith", ["split", "fp32"])
def test_fast_dstdgcb(name, arith):
    d = load_npz("dstdgcn_fast.npz")
    cin, cout, layout, T, V = BLOCKS[name]
    blk = _load(F.DSTDGCB(cin, cout, T, V, layout), group(d, f"{name}/sd/")).to(DEV).eval()
    blk.gc_arithmetic = arith
    with torch.no_grad():
        y = blk(t(d[f"{name}/x"]))
    assert y.shape == (1, T, V, cout)
    assert rel_err(y.cpu().numpy(), d[f"{name}/y64"]) <= 1e-4


@pytest.mark.parametrize("tag", ["h36m", "3dpw"])
@pytest.mark.parametrize("arith", ["split", "fp32"])
def test_fast_dstdgcn_fixture(tag, arith):
    d = load_npz("dstdgcn_fast.npz")
    m, _ = _model(tag, d)
    m.set_gc_arithmetic(arith)
    with torch.no_grad():
        y = m(t(d[f"model_{tag}/x"]))
    assert rel_err(y.cpu().numpy(), d[f"model_{tag}/y64"]) <= model_tol(d[f"model_{tag}/ref32_err"])


def test_fast_dstdgcn_batch256_vs_oracle():
    """B=256 (the bench batch) against the fp64 fast oracle on a subset, and
    every sample equal to its own B=1 forward (bit-exact)."""
    d = load_npz("dstdgcn_fast.npz")
    m, opts = _model("h36m", d)
    g = torch.Generator().manual_seed(7)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = torch.randn(256, T, 22, 3, generator=g)
    x[:, 10:] = x[:, 9:10]
    with torch.no_grad():
        y = m(x.to(DEV)).cpu()
        y1 = torch.cat([m(x[i:i + 1].to(DEV)).cpu() for i in (0, 77, 255)])
    assert torch.equal(y1, y[[0, 77, 255]])
    sd = group(d, "model_h36m/sd/")
    idx = [0, 1, 128, 255]
    y64 = O.fast_dstdgcn(x[idx], sd, 5).numpy()
    y32 = O.fast_dstdgcn(x[idx], sd, 5, dtype=torch.float32).numpy()
    assert rel_err(y[idx].numpy(), y64) <= model_tol(rel_err(y32, y64))


def test_fast_schema_and_cache():
    """The shadow is no part of state_dict / parameters; an in-place weight
    update, a write through .data (+ invalidate_native_cache) and a
    load_state_dict are all seen by the next forward; a deepcopy runs alone."""
    d = load_npz("dstdgcn_fast.npz")
    m, opts = _model("h36m", d)
    keys = list(m.state_dict())
    x = t(d["model_h36m/x"])
    with torch.no_grad():
        y0 = m(x)
    assert list(m.state_dict()) == keys and len(keys) == len(group(d, "model_h36m/sd/"))
    assert all(not k.startswith("_shadow") for k in keys)
    w = m.encoders[2][0].stgcn[0][0].conv_t[0].conv_rm.weight
    with torch.no_grad():
        w.mul_(2.0)
        y1 = m(x)
        fresh = copy.deepcopy(m)
        assert torch.equal(fresh(x), y1)
        w.data.mul_(0.5)  # exact: the original weights
        invalidate_native_cache(m)
        y2 = m(x)
    assert not torch.equal(y0, y1)
    assert torch.equal(y2, y0)
    m2 = F.DSTDGCN(**opts).to(DEV).eval()
    m2.load_state_dict(m.state_dict())
    with torch.no_grad():
        assert torch.equal(m2(x), y2)


@pytest.mark.parametrize("paired", [False, True])
def test_fast_train_step_vs_reference_fp64(paired):
    """One training step (forward + inverse pass, two losses, backward) of the
    fast model in train mode -- two calls, or one forward_pair -- loss, every
    gradient and the BN running-stat updates against the reference's fp64 run
    (dstdgcn_fast.npz train/*)."""
    from engine import mpjpe_error_3d
    d = load_npz("dstdgcn_fast.npz")
    opts = {k[len("train/opt/"):]: d[k].item() for k in d.files if k.startswith("train/opt/")}
    sd0 = group(d, "train/sd0/")
    m = _load(F.DSTDGCN(**opts), sd0).to(DEV).train()
    inp, inv, seq = (t(d[f"train/{n}"]) for n in ("inp", "inv", "seq"))
    B, T, VC = inp.shape
    V = VC // 3
    if paired:
        y, y_i = m.forward_pair(inp.view(B, T, V, 3), inv.view(B, T, V, 3))
    else:
        y, y_i = m(inp.view(B, T, V, 3)), m(inv.view(B, T, V, 3))
    loss = mpjpe_error_3d(y.reshape(B, T, VC), seq)
    loss_i = mpjpe_error_3d(y_i.reshape(B, T, VC), seq.flip(1))
    all_loss = (loss + loss_i) / 2
    all_loss.backward()
    assert abs(float(all_loss.detach()) - float(d["train/loss64"])) / float(d["train/loss64"]) < 1e-5
    # running statistics (two train forwards, momentum 0.1) and the batch counter
    sd = m.state_dict()
    for k in (k for k in d.files if k.startswith("train/sd1/")):
        name = k[len("train/sd1/"):]
        assert rel_err(sd[name].cpu().numpy(), d[k]) <= 1e-4, name
    assert int(sd["bn_in.bn.num_batches_tracked"]) == int(sd0["bn_in.bn.num_batches_tracked"]) + 2
    # gradients: error over the fp32 noise of the reference and of the fp32 oracle
    P = {k: torch.tensor(v, dtype=torch.float32, requires_grad=not k.endswith(("A_t", "running_mean", "running_var")))
         for k, v in sd0.items() if not k.endswith("num_batches_tracked")}
    outs = [O.fast_dstdgcn_fn(torch.from_numpy(d[f"train/{n}"]).view(B, T, V, 3), P, opts["num_layers"],
                              training=True).reshape(B, T, VC) for n in ("inp", "inv")]
    seq_c = torch.from_numpy(d["train/seq"])
    ((O.mpjpe_error_3d(outs[0], seq_c) + O.mpjpe_error_3d(outs[1], seq_c.flip(1))) / 2).backward()
    named = dict(m.named_parameters())
    keys = [k[len("train/g64/"):] for k in d.files if k.startswith("train/g64/")]
    assert set(keys) == {k for k, p in named.items() if p.requires_grad}
    ratios = []
    for k in keys:
        ref = d["train/g64/" + k].astype(np.float64)
        scale = float(np.abs(ref).max())
        noise = max(float(d["train/g32err/" + k]), float(np.abs(P[k].grad.double().numpy() - ref).max()),
                    1e-4 * scale)
        err = float(np.abs(named[k].grad.double().cpu().numpy() - ref).max())
        ratios.append((err / noise, k))
    ratios.sort(reverse=True)
    r = np.array([x[0] for x in ratios])
    assert np.median(r) <= 1.5, (np.median(r), ratios[:8])
    assert np.quantile(r, 0.9) <= 3.0, (np.quantile(r, 0.9), ratios[:8])
    # the tail is the global-sum gradients (PReLU slopes, alphas, biases in
    # front of BN), as in test_model_step_gradients_vs_reference_fp64; this
    # fixture's B=4 batch sums fewer terms than its B=8 (tail measured 12.6x)
    assert r.max() <= 16.0, ratios[:8]


def test_fast_op_and_block_gradients_vs_oracle():
    """Autograd through a single fast DSTDGC (incl. dA, dalpha, dx) and a
    train-mode fast DSTDGCB against fp64 autograd on the oracle."""
    d = load_npz("dstdgcn_fast.npz")
    for name in ("op_s_64_64", "op_t_64_64"):
        mode, cin, cout, T, V = OPS[name]
        ref, kpt = (T, V) if mode == "spatial" else (V, T)
        sd = group(d, f"{name}/sd/")
        op = _load(F.DSTDGC(cin, cout, ref, kpt, mode=mode), sd).to(DEV)
        x = t(d[f"{name}/x"]).requires_grad_()
        A = t(d[f"{name}/A"]).requires_grad_()
        al = t(d[f"{name}/alpha"]).requires_grad_()
        gy = torch.randn(1, T, V, cout, generator=torch.Generator().manual_seed(3))
        (op(x, A, al) * gy.to(DEV)).sum().backward()
        P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in sd.items()}
        x64 = torch.tensor(d[f"{name}/x"], dtype=torch.float64, requires_grad=True)
        A64 = torch.tensor(d[f"{name}/A"], dtype=torch.float64, requires_grad=True)
        a64 = torch.tensor(d[f"{name}/alpha"], dtype=torch.float64, requires_grad=True)
        (O.fast_dstdgc(x64, P, A64, a64.reshape(()), mode) * gy.double()).sum().backward()
        named = dict(op.named_parameters())
        for k, p in P.items():
            assert rel_err(named[k].grad.cpu().numpy(), p.grad.numpy()) <= 1e-4, (name, k)
        for got, want in ((x.grad, x64.grad), (A.grad, A64.grad), (al.grad, a64.grad)):
            assert rel_err(got.cpu().numpy(), want.numpy()) <= 1e-4, name
    name = "blk_64_64"
    cin, cout, layout, T, V = BLOCKS[name]
    sd = group(d, f"{name}/sd/")
    blk = _load(F.DSTDGCB(cin, cout, T, V, layout), sd).to(DEV).train()
    xb = torch.randn(4, T, V, cin, generator=torch.Generator().manual_seed(5))
    gy = torch.randn(4, T, V, cout, generator=torch.Generator().manual_seed(6))
    x = xb.to(DEV).requires_grad_()
    (blk(x) * gy.to(DEV)).sum().backward()
    P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=not k.endswith(("A_t", "running_mean",
                                                                                "running_var")))
         for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    x64 = xb.double().requires_grad_()
    (O.fast_dstdgcb(x64, P, training=True) * gy.double()).sum().backward()
    named = dict(blk.named_parameters())
    for k, p in P.items():
        if p.requires_grad:
            assert rel_err(named[k].grad.cpu().numpy(), p.grad.numpy()) <= 2e-4, k
    assert rel_err(x.grad.cpu().numpy(), x64.grad.numpy()) <= 2e-4


def test_fast_eval_mode_backward():
    """An eval-mode fast model under autograd: gradients reach the fast
    parameters (through the derivation) and equal the fast oracle's fp64
    autograd within the fp32 noise band; running statistics untouched."""
    d = load_npz("dstdgcn_fast.npz")
    m, opts = _model("h36m", d)
    before = {k: v.clone() for k, v in m.state_dict().items() if "running_" in k or "num_batches" in k}
    x = t(d["model_h36m/x"]).requires_grad_()
    y = m(x)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(13))
    (y * gy.to(DEV)).sum().backward()
    assert all(torch.equal(m.state_dict()[k], v) for k, v in before.items())
    sd = group(d, "model_h36m/sd/")

    def oracle(dtype, device="cpu"):
        P = {k: torch.tensor(v, dtype=dtype, device=device) for k, v in sd.items()
             if not k.endswith("num_batches_tracked")}
        for k, v in P.items():
            if not k.endswith(("A_t", "running_mean", "running_var")):
                v.requires_grad_(True)
        xo = torch.tensor(d["model_h36m/x"], dtype=dtype, device=device)
        (O.fast_dstdgcn_fn(xo, P, 5) * gy.to(device, dtype)).sum().backward()
        return P

    # fp32 noise of two other implementations: the oracle on the CPU and on the GPU (torch-ROCm ops)
    P, P32s = oracle(torch.float64), (oracle(torch.float32), oracle(torch.float32, DEV))
    named = dict(m.named_parameters())
    r = []
    for k, p in P.items():
        if p.requires_grad:
            ref = p.grad.numpy()
            noise = max(max(float(np.abs(Q[k].grad.double().cpu().numpy() - ref).max()) for Q in P32s),
                        1e-4 * float(np.abs(ref).max()))
            r.append((float(np.abs(named[k].grad.double().cpu().numpy() - ref).max()) / noise, k))
    r.sort(reverse=True)
    v = np.array([a for a, _ in r])
    assert np.median(v) <= 1.5 and np.quantile(v, 0.9) <= 3.0, r[:8]
    from test_gpu_train import check_tail
    check_tail(r)


def test_fast_model_in_the_engine():
    """engine.PredictionEngine trains the fast variant unchanged: the first
    epoch's loss equals the fp64 fast oracle's (train-mode BN), the loss falls
    over three one-batch epochs, Adam moves the fast parameters (through the
    derivation) and the batch counters advance once per forward."""
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    d = load_npz("dstdgcn_fast.npz")
    opts = {k[len("train/opt/"):]: d[k].item() for k in d.files if k.startswith("train/opt/")}
    sd0 = group(d, "train/sd0/")
    m = _load(F.DSTDGCN(**opts), sd0).to(DEV)
    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    eng = PredictionEngine(cfg, m, _Log())
    inp, inv, seq = (torch.from_numpy(d[f"train/{n}"]) for n in ("inp", "inv", "seq"))
    B, T, VC = inp.shape
    w0 = m.encoders[0][0].stgcn[0][0].conv_s[0].conv_f.weight.detach().clone()
    losses = [eng.train([(inp, inv, seq, seq)], s, max_iter=1) for s in range(3)]
    y64 = O.fast_dstdgcn(inp.view(B, T, VC // 3, 3), sd0, opts["num_layers"], training=True).reshape(B, T, VC)
    l64 = float(O.mpjpe_error_3d(y64, seq.double()))
    assert abs(losses[0] - l64) / l64 < 1e-5, (losses[0], l64)
    assert np.isfinite(losses).all() and losses[-1] < losses[0]
    assert not torch.equal(w0, m.encoders[0][0].stgcn[0][0].conv_s[0].conv_f.weight.detach())
    assert int(m.bn_in.bn.num_batches_tracked) == int(sd0["bn_in.bn.num_batches_tracked"]) + 6
