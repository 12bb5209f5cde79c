"""MI355X parity of the training path: native train-mode
forward + backward vs autograd through the CPU oracle in fp64, which
tests/test_oracle_golden.py pins to the reference's own fp64 gradients and
loss curve (train_grads.npz).

Tolerances
  single DSTDGC op        : every output / gradient within 1e-4 of its max |ref|
  DSTDGCB (train-mode BN) : 2e-4 (BN backward subtracts two O(1) means)
  whole model, one step   : err / noise per tensor, where noise is the largest
                            fp32 error of ten other fp32 runs (the oracle's
                            fp32 step on the CPU, on the GPU and over 8 sample
                            orders, plus the reference's g32err where the
                            fixture holds it) -- the 21-op stack is chaotic in
                            fp32: every tensor within 3x, the
                            global sums within 4x (bars calibrated by
                            leave-one-out over those runs,
                            profiles/r06g_grad_bar_calibration.json), median
                            <= 1.5, 90th percentile <= 2 (fp32_noise /
                            check_ratios; the per-block bisection behind it:
                            test_model_step_gradient_tail_is_propagation)
  eval-mode model backward: the former two-sample criterion (GLOBAL_SUM /
                            check_tail, below)
  5-step loss curve       : within twice the reference's own fp32 deviation
                            from its fp64 curve
"""
import os

import re

import numpy as np
import pytest
import torch

import dstd_native as native
from conftest import group, load_npz
from model import DSTDGC, DSTDGCB, get_model
from oracle import dstdgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, ref):
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.as_tensor(a, dtype=torch.float64)
    ref = ref.detach().double().cpu() if torch.is_tensor(ref) else torch.as_tensor(ref, dtype=torch.float64)
    return float((a - ref).abs().max() / max(float(ref.abs().max()), 1e-30))


def randomise(module, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith(("A_s", "A_t")):
                continue
            if p.dim() == 1 and p.numel() == 1:  # alphas, PReLU slopes
                p.copy_(torch.empty(1).uniform_(0.2, 0.8, generator=g))
            elif name.endswith("bias") or p.dim() == 1:
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith(("W_s", "R_t")):
                p.copy_(0.2 * torch.randn(p.shape, generator=g))
            elif name.endswith("R_s"):
                p.add_(0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("bn.weight"):
                p.copy_(torch.empty(p.shape).uniform_(0.8, 1.2, generator=g))


# ---- single DSTDGC ---------------------------------------------------------
OPS = [("spatial", 64, 64, 35, 22), ("spatial", 6, 64, 35, 22), ("spatial", 64, 3, 40, 23),
       ("temporal", 64, 64, 35, 22), ("temporal", 3, 3, 40, 23), ("temporal", 64, 64, 75, 22),
       ("spatial", 32, 48, 20, 17), ("temporal", 48, 32, 20, 17)]


@pytest.mark.parametrize("mode,cin,cout,T,V", OPS)
def test_dstdgc_op_backward(mode, cin, cout, T, V):
    torch.manual_seed(cin * 7 + T)
    ref_c, kpt = (T, V) if mode == "spatial" else (V, T)
    op = DSTDGC(cin, cout, ref_c, kpt, mode=mode)
    randomise(op, cin + cout + T)
    NN = V if mode == "spatial" else T
    B = 3
    x = torch.randn(B, cin, T, V)
    A = 0.3 * torch.randn(1, NN, NN)
    alpha = torch.tensor([0.7])
    w = torch.randn(B, cout, T, V)
    # oracle (fp64 autograd)
    sd64 = {k: v.detach().double().requires_grad_(True) for k, v in op.state_dict().items()}
    x64, A64, a64 = (t.double().requires_grad_(True) for t in (x, A, alpha))
    y64 = O.dstdgc(x64, sd64, A64, a64.reshape(()), mode)
    (y64 * w.double()).sum().backward()
    # native
    op = op.to(DEV)
    xg, Ag, ag = (t.to(DEV).requires_grad_(True) for t in (x, A, alpha))
    y = op(xg, Ag, ag)
    assert y.grad_fn is not None
    (y * w.to(DEV)).sum().backward()
    assert rel(y, y64) < 1e-4
    assert rel(xg.grad, x64.grad) < 1e-4
    assert rel(Ag.grad, A64.grad) < 1e-4
    assert rel(ag.grad, a64.grad) < 1e-4
    for name, p in op.named_parameters():
        assert rel(p.grad, sd64[name].grad) < 1e-4, name


def test_dstdgc_op_backward_partial_row_tiles():
    """Spatial op with 40 output channels at B=64: the backward aggregation
    runs its 4-row-tile (64-channel) kernel over 40 channels with every wave
    busy (8 frames per workgroup on a 256-CU device: slab 196 floats per
    channel row, 100 KB of LDS sized for 64 rows), and the test checks that
    this kernel is the one that ran (dstd_debug_aggb_last); at B=128 the
    64-row slab would not fit and the dispatch takes the 16-channel kernel
    (reference model/dstdgcn.py:80-87 under autograd, fp64 oracle)."""
    mode, cin, cout, T, V, B = "spatial", 32, 40, 40, 23, 64
    torch.manual_seed(5)
    op = DSTDGC(cin, cout, T, V, mode=mode)
    randomise(op, 77)
    x = torch.randn(B, cin, T, V)
    A = 0.3 * torch.randn(1, V, V)
    alpha = torch.tensor([0.7])
    w = torch.randn(B, cout, T, V)
    sd64 = {k: v.detach().double().requires_grad_(True) for k, v in op.state_dict().items()}
    x64, A64, a64 = (t.double().requires_grad_(True) for t in (x, A, alpha))
    (O.dstdgc(x64, sd64, A64, a64.reshape(()), mode) * w.double()).sum().backward()
    op = op.to(DEV)
    xg, Ag, ag = (t.to(DEV).requires_grad_(True) for t in (x, A, alpha))
    (op(xg, Ag, ag) * w.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert native.lib().dstd_debug_aggb_last() == 64
    assert rel(xg.grad, x64.grad) < 1e-4
    assert rel(Ag.grad, A64.grad) < 1e-4
    for name, p in op.named_parameters():
        assert rel(p.grad, sd64[name].grad) < 1e-4, name


def test_aggb_dispatch_falls_back_to_16_channel_chunks():
    """Where the 64-channel slab of the spatial aggregation backward does not
    fit LDS (B=128 above; the model's H36M / 3DPW ops at B=256) the dispatch
    retries the 16-channel kernel before the two-launch path:
    the backward runs it and meets the same fp64 bar."""
    mode, cin, cout, T, V, B = "spatial", 32, 40, 40, 23, 128
    torch.manual_seed(6)
    op = DSTDGC(cin, cout, T, V, mode=mode)
    randomise(op, 78)
    x = torch.randn(B, cin, T, V)
    A = 0.3 * torch.randn(1, V, V)
    alpha = torch.tensor([0.7])
    w = torch.randn(B, cout, T, V)
    sd64 = {k: v.detach().double().requires_grad_(True) for k, v in op.state_dict().items()}
    x64, A64, a64 = (t.double().requires_grad_(True) for t in (x, A, alpha))
    (O.dstdgc(x64, sd64, A64, a64.reshape(()), mode) * w.double()).sum().backward()
    op = op.to(DEV)
    xg, Ag, ag = (t.to(DEV).requires_grad_(True) for t in (x, A, alpha))
    (op(xg, Ag, ag) * w.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert native.lib().dstd_debug_aggb_last() == 16
    assert rel(xg.grad, x64.grad) < 1e-4
    assert rel(Ag.grad, A64.grad) < 1e-4
    for name, p in op.named_parameters():
        assert rel(p.grad, sd64[name].grad) < 1e-4, name


@pytest.mark.parametrize("mode", ["spatial", "temporal"])
@pytest.mark.parametrize("red", [1, 3, 8])
def test_dstdgc_op_red_channels(mode, red):
    """DSTDGC(..., red_channels=R) (reference model/dstdgcn.py:55-68, any R):
    R P / Q channels, conv_rm over R*ref.  No-grad forward and backward both
    run the generic training kernels (the inference ones carry R = 2)."""
    torch.manual_seed(red)
    cin, cout, T, V = 32, 48, 35, 22
    ref_c, kpt = (T, V) if mode == "spatial" else (V, T)
    op = DSTDGC(cin, cout, ref_c, kpt, red_channels=red, mode=mode)
    assert op.conv_m1.weight.shape[0] == red and op.conv_rm.weight.shape[1] == red * ref_c
    randomise(op, 11 * red)
    NN = V if mode == "spatial" else T
    B = 3
    x = torch.randn(B, cin, T, V)
    A = 0.3 * torch.randn(1, NN, NN)
    alpha = torch.tensor([0.6])
    w = torch.randn(B, cout, T, V)
    sd64 = {k: v.detach().double().requires_grad_(True) for k, v in op.state_dict().items()}
    x64, A64, a64 = (t.double().requires_grad_(True) for t in (x, A, alpha))
    y64 = O.dstdgc(x64, sd64, A64, a64.reshape(()), mode)
    (y64 * w.double()).sum().backward()
    op = op.to(DEV)
    with torch.no_grad():
        y0 = op(x.to(DEV), A.to(DEV), alpha.to(DEV))
    assert rel(y0, y64) < 1e-4
    xg, Ag, ag = (t.to(DEV).requires_grad_(True) for t in (x, A, alpha))
    y = op(xg, Ag, ag)
    (y * w.to(DEV)).sum().backward()
    assert rel(y, y64) < 1e-4
    assert rel(xg.grad, x64.grad) < 1e-4
    assert rel(Ag.grad, A64.grad) < 1e-4
    assert rel(ag.grad, a64.grad) < 1e-4
    for name, p in op.named_parameters():
        assert rel(p.grad, sd64[name].grad) < 1e-4, name


@pytest.mark.parametrize("mode", ["spatial", "temporal"])
def test_fast_dstdgc_op_red_channels(mode):
    """The channels-last op (reference dstdgcn_fast.py:59-155) at R = 3."""
    from model.dstdgcn_fast import DSTDGC as FastDSTDGC
    torch.manual_seed(3)
    cin, cout, T, V = 16, 24, 40, 23
    ref_c, kpt = (T, V) if mode == "spatial" else (V, T)
    op = FastDSTDGC(cin, cout, ref_c, kpt, red_channels=3, mode=mode)
    randomise(op, 33)
    NN = V if mode == "spatial" else T
    x = torch.randn(2, T, V, cin)
    A = 0.3 * torch.randn(1, NN, NN)
    alpha = torch.tensor([0.6])
    sd = {k: v.detach().double() for k, v in op.state_dict().items()}
    y64 = O.fast_dstdgc(x.double(), sd, A.double(), alpha.double().reshape(()), mode)
    op = op.to(DEV)
    with torch.no_grad():
        y = op(x.to(DEV), A.to(DEV), alpha.to(DEV))
    assert rel(y, y64) < 1e-4


# ---- DSTDGCB in train mode ---------------------------------------------------
BLOCKS = [(6, 64, "h36m", 35, 22), (64, 64, "3dpw", 40, 23), (64, 3, "cmu", 35, 25),
          (64, 64, "h36m", 100, 22),  # T=100 ("50 in / 50 out"): generic kernels
          (64, 64, "h36m", 128, 22)]  # T=128: the envelope's top


@pytest.mark.parametrize("cin,cout,layout,T,V", BLOCKS)
def test_dstdgcb_train_forward_backward(cin, cout, layout, T, V):
    torch.manual_seed(cin + cout)
    blk = DSTDGCB(cin, cout, T, V, layout)
    randomise(blk, 100 + cin + cout)
    assert blk.A_s.data_ptr() == blk.R_s.data_ptr()
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    B = 4
    x = torch.randn(B, cin, T, V)
    w = torch.randn(B, cout, T, V)
    # oracle: A_s is a constant holding R_s's values (the alias)
    P = {k: v.double() for k, v in sd.items() if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    for k in P:
        if not k.endswith(("A_s", "A_t")):
            P[k].requires_grad_(True)
    P["A_s"] = P["R_s"].detach()
    x64 = x.double().requires_grad_(True)
    O.BN_RECORD = []
    y64 = O.dstdgcb(x64, P, training=True)
    stats = O.BN_RECORD
    O.BN_RECORD = None
    (y64 * w.double()).sum().backward()
    # native
    blk = blk.to(DEV).train()
    _realias(blk)
    xg = x.to(DEV).requires_grad_(True)
    y = blk(xg)
    (y * w.to(DEV)).sum().backward()
    tol = 2e-4
    assert rel(y, y64) < tol
    assert rel(xg.grad, x64.grad) < tol
    # a conv bias feeding a train-mode BN has a true gradient of ~0 (the BN
    # mean removes it): judge every tensor against the block's gradient scale
    gscale = max(float(P[k].grad.abs().max()) for k in P if P[k].grad is not None)
    for name, p in blk.named_parameters():
        if name == "A_s" or name == "A_t":
            assert p.grad is None
            continue
        ref = P[name].grad
        err = float((p.grad.double().cpu() - ref).abs().max())
        assert err <= tol * max(float(ref.abs().max()), 1e-3 * gscale), (name, err, float(ref.abs().max()))
    # running statistics: (1 - m) * old + m * batch (unbiased variance)
    bns = [m for m in blk.modules() if isinstance(m, torch.nn.BatchNorm1d)]
    assert len(bns) == len(stats)
    for bn, (mean, var) in zip(bns, stats):
        old_m = sd[[k for k in sd if k.endswith("running_mean") and bn is _bn_of(blk, k)][0]]
        old_v = sd[[k for k in sd if k.endswith("running_var") and bn is _bn_of(blk, k)][0]]
        assert rel(bn.running_mean, 0.9 * old_m.double() + 0.1 * mean) < 1e-5
        assert rel(bn.running_var, 0.9 * old_v.double() + 0.1 * var) < 1e-5
        assert int(bn.num_batches_tracked) == 1


def _bn_of(module, key):
    m = module
    for part in key.split(".")[:-1]:
        m = getattr(m, part)
    return m


# ---- whole model: one engine step vs the reference's fp64 gradients ---------
# The 21-op train-mode stack is ill-conditioned in fp32: a
# gradient's fp32 error is a draw from a wide distribution whose spread
# depends on the tensor (global sums such as alpha_sm are one sum over every
# position of both passes, cancelling ~5x10^4-fold on trained blocks:
# scripts/grad_tail_bisect.py, DESIGN.md section 8 "Gradient accuracy").  So
# the noise floor of each tensor is MEASURED as the largest fp32 error among
# several fp32 implementations / summation orders of the same step -- the
# fp32 oracle on the CPU, on the GPU (torch-ROCm ops), and on the GPU over
# N_ORDERS sample orders of the batch (the loss and train-mode BatchNorm are
# order-invariant, so each order is only another rounding sequence), plus the
# reference's own fp32 run where the fixture holds it -- and every tensor of
# the native step must be within MAX_RATIO of that floor (median <= 1.5,
# 90th percentile <= 2).  Before round 5 the floor was the max of two
# samples, and a tail exemption (12x for global sums) covered its undershoot.
# The largest-ratio bars are calibrated, not chosen (round 6,
# scripts/grad_bar_calibration.py, profiles/r06g_grad_bar_calibration.json):
# each fp32 run measured the way the native step is -- against the floor of
# the OTHER runs -- on the fixture step, B=32 and B=256 (31 leave-one-out
# runs), split by tensor class:
#  * every tensor but the global sums: largest ratio p95 2.22, max 2.71 ->
#    MAX_RATIO 3.0 (the native steps: at most 1.22);
#  * GLOBAL_SUM tensors (scalars and biases: ONE sum over every position of
#    both passes): p95 2.66, max 2.96.  The native step exceeds that on one
#    tensor per step at most -- B=32 3.17 (a block PReLU slope), the world-2
#    SyncBN step 3.40 (a conv_rm bias) -- which the per-block bisection
#    (test_model_step_gradient_tail_is_propagation, r05f) places in the
#    propagation through the 21-op chain, not in a kernel's summation (the
#    slope's partials carried in fp64 changed nothing, r06f) -> their bar
#    stays MAX_RATIO_GLOBAL 4.0, 1.35x the calibrated maximum.
N_ORDERS = 8
MAX_RATIO = 3.0
MAX_RATIO_GLOBAL = 4.0


def fp32_noise(sd0, batch, g64, extra=None, n_orders=N_ORDERS):
    """Per tensor: the largest |g32 - g64| over the fp32 oracle step on the
    CPU, on the GPU and on the GPU over n_orders sample orders of ``batch``
    (numpy (inp, inv, seq)); ``extra``: more per-tensor fp32 errors (the
    reference's own, train_grads.npz g32err)."""
    B = batch[0].shape[0]
    runs = [("cpu", None), (DEV, None)] + [(DEV, np.random.default_rng(s).permutation(B))
                                           for s in range(1, n_orders + 1)]
    noise = {k: float(extra[k]) if extra is not None else 0.0 for k in g64}
    for dev, perm in runs:
        P = O.train_params(sd0, torch.float32, dev)
        _, lall = O.step_loss(P, batch if perm is None else tuple(x[perm] for x in batch), 5)
        lall.backward()
        for k, v in P.items():
            if v.grad is not None:
                noise[k] = max(noise[k], float(np.abs(v.grad.double().cpu().numpy() - g64[k]).max()))
    return noise


def noise_ratios(grads, g64, noise):
    """(|g - g64|_max / max(noise, 1e-4 |g64|_max), tensor) for every tensor of g64."""
    out = []
    for k, r64 in g64.items():
        g = grads[k].double().cpu().numpy() if torch.is_tensor(grads[k]) else grads[k]
        scale = float(np.abs(r64).max())
        out.append((float(np.abs(g - r64).max()) / max(noise[k], 1e-4 * scale), k))
    return out


def check_ratios(ratios, what=""):
    r = np.array(sorted((v for v, _ in ratios), reverse=True))
    top = sorted(ratios, reverse=True)[:6]
    print(f"{what} err / fp32 noise floor: median {np.median(r):.2f}, p90 {np.quantile(r, 0.9):.2f}, "
          f"max {r[0]:.2f}", [(round(v, 2), k) for v, k in top[:3]])
    assert np.median(r) <= 1.5, (what, np.median(r), top)
    assert np.quantile(r, 0.9) <= 2.0, (what, np.quantile(r, 0.9), top)
    other = [(v, k) for v, k in ratios if not GLOBAL_SUM.search(k)]
    assert max(other)[0] <= MAX_RATIO, (what, sorted(other, reverse=True)[:3])
    assert r[0] <= MAX_RATIO_GLOBAL, (what, top)


# The eval-mode backward tests (tests/test_gpu_parity.py, test_gpu_fast.py;
# running-statistics BatchNorm, a random upstream gradient) keep the former
# two-sample criterion: every tensor above 3x must be a global sum
# (GLOBAL_SUM: the scalars and conv biases), those within 12x.
GLOBAL_SUM = re.compile(r"(alpha_sm|alpha_tm|prelu\.weight|encoders\.\d+\.2\.weight|"
                        r"conv_(f|m1|m2|rm)\.bias|residual\.0\.bias)$")


def check_tail(ratios, bar=3.0, global_bar=12.0):
    above = sorted(((v, k) for v, k in ratios if v > bar), reverse=True)
    print(f"gradient error / fp32 noise above {bar}x ({len(above)} of {len(ratios)}):",
          [(round(v, 2), k) for v, k in above])
    assert all(GLOBAL_SUM.search(k) for _, k in above), [(v, k) for v, k in above if not GLOBAL_SUM.search(k)]
    assert all(v <= global_bar for v, _ in above), above[:4]


def _realias(model):
    """Module.to() converts each parameter separately and so splits the
    A_s/R_s storage alias (the reference's runner does the same with
    model.to(device), runner/base.py:34-35).  The fixtures were produced on
    the CPU with the alias intact; restore it to compare like with like."""
    for m in model.modules():
        if isinstance(m, DSTDGCB):
            m.A_s.data = m.R_s.data


def _model_3dpw():
    d = load_npz("engine.npz")
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "train/sd0/").items()})
    m = m.to(DEV)
    _realias(m)
    return m.train(), d


def test_model_step_gradients_vs_reference_fp64():
    from engine import mpjpe_error_3d
    m, d = _model_3dpw()
    g = load_npz("train_grads.npz")
    inp, inv, seq = (torch.from_numpy(d[f"train/{n}0"]).to(DEV) for n in ("inp", "inv", "seq"))
    B, T, VC = inp.shape
    out = m(inp.view(B, T, 23, 3)).view(B, T, VC)
    out_i = m(inv.view(B, T, 23, 3)).view(B, T, VC)
    loss = mpjpe_error_3d(out, seq)
    all_loss = (loss + mpjpe_error_3d(out_i, seq.flip(1))) / 2
    all_loss.backward()
    assert abs(float(loss) - float(d["train/losses"][0])) / float(d["train/losses"][0]) < 1e-5
    named = dict(m.named_parameters())
    keys = [k[4:] for k in g.files if k.startswith("g64/")]
    assert set(keys) == {k for k, p in named.items() if p.requires_grad}
    g64 = {k: g["g64/" + k] for k in keys}
    noise = fp32_noise(group(d, "train/sd0/"), tuple(d[f"train/{n}0"] for n in ("inp", "inv", "seq")), g64,
                       extra={k: g["g32err/" + k] for k in keys})
    check_ratios(noise_ratios({k: named[k].grad for k in keys}, g64, noise), "fixture step (two calls)")
    assert named["conv_st_in.stgcn.0.0.A_s"].grad is None


@pytest.mark.parametrize("B", [32, 256])
def test_model_step_gradients_at_training_batch(B):
    """One engine step the way PredictionEngine.train runs it (forward_pair
    over the batch and its time reversal, two mpjpe losses, the native
    backward into the in-place gradient arena; engine/prediction.py:231-294)
    at the yaml's train_batch_size, 32 (configs/dstdgcn/dstdgcn_3dpw.yaml:19),
    and at 256: the reduce GEMMs pick their split-K partition from the sample
    count, so these batches run other partitions than the fixture's B=8.
    Reference: the oracle's fp64 step (pinned to the reference's own fp64
    gradients by tests/test_oracle_golden.py); fp32 noise: the oracle's fp32
    step as torch ops on the GPU (rocBLAS) and on the CPU -- the same
    per-tensor criterion as the B=8 fixture step."""
    from engine import mpjpe_error_3d
    m, d = _model_3dpw()
    m._dstd_inplace_grads = True
    g = torch.Generator().manual_seed(1000 + B)
    T, VC = 40, 69
    seq = 0.6 * torch.randn(B, T, VC, generator=g)  # the fixture batches' scale
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]  # future frames = the last observed one
    rev = seq.flip(1)
    inv = rev.clone()
    inv[:, 10:] = inv[:, 9:10]
    batch = (inp.numpy(), inv.numpy(), seq.numpy())
    # native
    sq = seq.to(DEV)
    p1, p2 = m.forward_pair(inp.view(B, T, 23, 3).to(DEV), inv.view(B, T, 23, 3).to(DEV))
    loss = mpjpe_error_3d(p1.reshape(B, T, VC), sq)
    all_loss = (loss + mpjpe_error_3d(p2.reshape(B, T, VC), sq.flip(1))) / 2
    all_loss.backward()
    # the oracle's fp64 step and the fp32 noise floor
    sd0 = group(d, "train/sd0/")
    P = O.train_params(sd0, torch.float64, DEV)
    l0, lall = O.step_loss(P, batch, 5)
    lall.backward()
    g64 = {k: v.grad.double().cpu().numpy() for k, v in P.items() if v.grad is not None}
    assert abs(float(loss.detach()) - float(l0)) / float(l0) < 1e-5
    named = dict(m.named_parameters())
    assert set(g64) == {k for k, p in named.items() if p.requires_grad}
    noise = fp32_noise(sd0, batch, g64)
    check_ratios(noise_ratios({k: named[k].grad for k in g64}, g64, noise), f"B={B} step")


def test_wgrad_stream_is_bit_identical():
    """The model backward's weight-gradient stream (each DSTDGC's dW_rm and
    packed-conv weight reductions forked onto a second HIP stream, alternating
    dG / dD buffer sets; dstd_train_capi.hip WgradStream) against every launch
    on the caller's stream (DSTD_TRAIN_ONE_STREAM): the same step at the
    training batch gives bit-identical gradients and input gradient, three
    times over (a missing fork / release / join shows up as a difference)."""
    from engine import mpjpe_error_3d
    m, _ = _model_3dpw()
    g = torch.Generator().manual_seed(77)
    B, T, VC = 32, 40, 69
    seq = (0.6 * torch.randn(B, T, VC, generator=g)).to(DEV)
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]

    def step(one_stream):
        m._dstd_one_stream = one_stream
        m.zero_grad(set_to_none=True)
        x = inp.view(B, T, 23, 3).clone().requires_grad_(True)
        loss = mpjpe_error_3d(m(x).reshape(B, T, VC), seq)
        loss.backward()
        return [p.grad.clone() for p in m.parameters() if p.grad is not None] + [x.grad.clone()]

    with torch.random.fork_rng(devices=[DEV]):
        ref = step(True)
    for _ in range(3):
        with torch.random.fork_rng(devices=[DEV]):
            got = step(False)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)
    m._dstd_one_stream = False


@pytest.mark.parametrize("inplace", [True, False])
def test_forward_pair_equals_two_calls(inplace):
    """DSTDGCN.forward_pair (DSTD_TRAIN_PAIRED: one launch sequence over the
    batch and its time reversal, BatchNorm statistics per half, running
    statistics updated by the first half then the second) against the two
    train-mode calls of engine/prediction.py:231-287: outputs, every gradient,
    running statistics and num_batches_tracked.  The paths differ only in
    GEMM summation order (split-K over 64 samples vs 32 + 32)."""
    from engine import mpjpe_error_3d
    m1, d = _model_3dpw()
    m2, _ = _model_3dpw()
    m1._dstd_inplace_grads = m2._dstd_inplace_grads = inplace
    inp, inv, seq = (torch.from_numpy(d[f"train/{n}0"]).to(DEV) for n in ("inp", "inv", "seq"))
    B, T, VC = inp.shape
    x1, x2 = inp.view(B, T, 23, 3), inv.view(B, T, 23, 3)

    def loss_of(o1, o2):
        return (mpjpe_error_3d(o1.reshape(B, T, VC), seq) + mpjpe_error_3d(o2.reshape(B, T, VC), seq.flip(1))) / 2

    y1, y2 = m1(x1), m1(x2)
    loss_of(y1, y2).backward()
    p1, p2 = m2.forward_pair(x1, x2)
    loss_of(p1, p2).backward()
    assert rel(p1, y1) < 1e-5 and rel(p2, y2) < 1e-5
    for (name, a), b in zip(m1.named_parameters(), m2.parameters()):
        if a.grad is None:
            assert b.grad is None, name
            continue
        if name.endswith("residual.0.bias"):
            # analytically zero (the train-mode BN right after it cancels a
            # per-channel constant): both paths hold fp32 rounding noise
            assert float(b.grad.abs().max()) < 1e-3, name
            continue
        assert float((a.grad - b.grad).abs().max()) <= 1e-4 * float(a.grad.abs().max()) + 1e-12, name
    for (name, a), b in zip(m1.named_buffers(), m2.buffers()):
        if name.endswith("num_batches_tracked"):
            assert int(a) == int(b) == 2, name
        else:
            assert rel(b, a) < 1e-5, name
    # eval mode: the two plain calls
    m2.eval()
    with torch.no_grad():
        e1, e2 = m2.forward_pair(x1, x2)
        assert torch.equal(e1, m2(x1)) and torch.equal(e2, m2(x2))


def test_gradient_sink_paths_agree():
    """The model backward accumulates into the parameters' .grad in place
    (dstd_native.grad_sink) when they are its own arena views, and hands
    fresh views to autograd otherwise: both give the same gradients, a second
    backward without zero_grad accumulates (torch semantics), and the
    gradients of a step with the inverse pass are slices of one buffer."""
    from engine import mpjpe_error_3d
    m, d = _model_3dpw()
    inp, inv, seq = (torch.from_numpy(d[f"train/{n}0"]).to(DEV) for n in ("inp", "inv", "seq"))
    B, T, VC = inp.shape

    def step():
        out = m(inp.view(B, T, 23, 3)).view(B, T, VC)
        out_i = m(inv.view(B, T, 23, 3)).view(B, T, VC)
        ((mpjpe_error_3d(out, seq) + mpjpe_error_3d(out_i, seq.flip(1))) / 2).backward()

    # the paths differ only in summation order (arena += vs autograd's sum of
    # two arenas): 1e-4 of a tensor's max covers the global-sum scalars
    # (alphas, PReLU slopes, ~1e-5 measured), far inside their fp32 noise
    TOL = 1e-4
    params = [p for p in m.parameters() if p.requires_grad]
    m._dstd_inplace_grads = True  # what engine.PredictionEngine.train opts into
    # in-place mode: one anchor leaf stands in for the ~300 parameters as the
    # Function's tensor inputs (x, anchor -- dstdgcn._anchor_of)
    probe = m(inp.view(B, T, 23, 3))
    assert len(probe.grad_fn.next_functions) == 2, len(probe.grad_fn.next_functions)
    del probe
    m._dstd_inplace_grads = False
    probe = m(inp.view(B, T, 23, 3))
    assert len(probe.grad_fn.next_functions) == 1 + len(list(m.parameters()))
    del probe
    m._dstd_inplace_grads = True
    step()  # direct: .grad were None
    g_direct = [p.grad.clone() for p in params]
    bases = {p.grad._base.data_ptr() for p in params}
    assert len(bases) == 1 and all(p.grad._base is not None for p in params)
    step()  # no zero_grad: accumulates into the same views
    for p, g in zip(params, g_direct):
        assert float((p.grad - 2 * g).abs().max()) <= TOL * float(g.abs().max()) + 1e-12
    for p in params:  # user-owned gradients: the autograd path
        p.grad = torch.zeros_like(p)
    step()
    for p, g in zip(params, g_direct):
        assert p.grad._base is None
        assert float((p.grad - g).abs().max()) <= TOL * float(g.abs().max()) + 1e-12
    m.zero_grad(set_to_none=True)
    step()  # back to the in-place arena
    assert all(p.grad._base is not None for p in params)
    # a parameter hook (DDP, user hooks) turns the in-place path off ...
    m.zero_grad(set_to_none=True)
    h = params[0].register_hook(lambda g: g)
    step()
    h.remove()
    assert all(p.grad._base is None for p in params)
    for p, g in zip(params, g_direct):
        assert float((p.grad - g).abs().max()) <= TOL * float(g.abs().max()) + 1e-12
    # ... and so does not opting in (the default for every caller but the engine)
    m._dstd_inplace_grads = False
    m.zero_grad(set_to_none=True)
    step()
    assert all(p.grad._base is None for p in params)
    grads = torch.autograd.grad(  # autograd.grad sees the gradients and leaves .grad alone
        mpjpe_error_3d(m(inp.view(B, T, 23, 3)).view(B, T, VC), seq), params)
    assert all(g is not None for g in grads)


def test_autocast_bf16_runs_the_fp32_path():
    """Config 5 names a bf16 training loop: under torch.autocast(bf16) the
    native model computes in fp32 (arithmetic >= bf16; autocast does not
    retype custom autograd Functions), so loss and gradients equal the plain
    fp32 step bit for bit."""
    from engine import mpjpe_error_3d
    m, d = _model_3dpw()
    inp, seq = (torch.from_numpy(d[f"train/{n}0"]).to(DEV) for n in ("inp", "seq"))
    B, T, VC = inp.shape
    res = []
    for ac in (False, True):
        m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "train/sd0/").items()})
        _realias(m)
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
            out = m(inp.view(B, T, 23, 3)).view(B, T, VC)
            loss = mpjpe_error_3d(out, seq)
        assert out.dtype == torch.float32
        loss.backward()
        res.append((float(loss), [p.grad.clone() for p in m.parameters() if p.requires_grad]))
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


def test_training_curve_matches_reference():
    """PredictionEngine.train, 5 one-batch epochs on the engine.npz 3DPW run."""
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    m, d = _model_3dpw()
    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    eng = PredictionEngine(cfg, m, _Log())
    batches = [tuple(torch.from_numpy(d[f"train/{n}{i}"]) for n in ("inp", "inv", "seq", "seq")) for i in range(4)]
    losses = np.array([eng.train([batches[s % 4]], s, max_iter=1) for s in range(5)])
    c64 = load_npz("train_grads.npz")["losses64"]
    ref32 = d["train/losses"]
    band = np.abs(ref32 - c64).max() / c64.max()
    assert abs(losses[0] - c64[0]) / c64[0] < 1e-5
    assert np.abs(losses - c64).max() / c64.max() <= 2 * band, (losses, c64, ref32)
    assert losses[-1] < 0.75 * losses[0]
    # A_s still aliases R_s after Adam updated R_s in place
    blk = m.conv_st_in.stgcn[0][0]
    assert blk.A_s.data_ptr() == blk.R_s.data_ptr()


def test_graphed_engine_step_equals_eager():
    """learn.graph: the engine's step captured as a HIP graph (engine/graphed.py)
    and replayed -- after the warm-up is undone, replay k is eager step k bit
    for bit (the same capturable Adam both ways), across StepLR boundaries
    (the tensor learning rate updated in place) and a ragged last batch that
    runs eagerly; and the replays really are graph launches."""
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    d = load_npz("engine.npz")
    batches = [tuple(torch.from_numpy(d[f"train/{n}{i}"]) for n in ("inp", "inv", "seq", "seq")) for i in range(4)]
    ragged = tuple(t[:6] for t in batches[3])
    engines = []
    for graphed in (True, False):
        m, _ = _model_3dpw()
        cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.5, step_size=2, graph=True),
                   loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
        eng = PredictionEngine(cfg, m, _Log())
        if not graphed:
            eng._graphed = lambda: False  # same capturable Adam, eager steps
        losses = [eng.train(batches[:3] + [ragged], e) for e in range(3)]
        engines.append((eng, m, losses))
    (eg, mg, lg), (ee, me, le) = engines
    assert eg._graph_step is not None and ee._graph_step is None
    assert lg == le, (lg, le)
    for (n, a), b in zip(mg.named_parameters(), me.parameters()):
        assert torch.equal(a, b), n
    for (n, a), b in zip(mg.named_buffers(), me.buffers()):
        assert torch.equal(a, b), n
    lr_g, lr_e = (float(e.optimizer.param_groups[0]["lr"]) for e in (eg, ee))
    assert lr_g == lr_e and abs(lr_g - 1.5e-3) < 1e-9, (lr_g, lr_e)
    assert lg[-1] < lg[0]


def test_graphed_engine_test_after_replays():
    """learn.graph with epochs made only of replays (one full batch): a replay
    updates parameters and BatchNorm buffers on the device without moving
    their version counters, so test() after it must not reuse the BatchNorm
    constants the previous test() folded (engine/graphed.py invalidates the
    native cache after every replay).  Every epoch's metric equals the eager
    engine's bit for bit."""
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    d = load_npz("engine.npz")
    batch = tuple(torch.from_numpy(d[f"train/{n}0"]) for n in ("inp", "inv", "seq", "seq"))
    g = torch.Generator().manual_seed(7)
    all_seqs = 0.6 * torch.randn(6, 40, 69, generator=g)
    inputs = all_seqs.clone()
    inputs[:, 10:] = inputs[:, 9:10]
    loader = [(inputs, None, None, all_seqs)]
    runs = []
    for graphed in (True, False):
        m, _ = _model_3dpw()
        cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.5, step_size=2, graph=True),
                   loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
        eng = PredictionEngine(cfg, m, _Log())
        if not graphed:
            eng._graphed = lambda: False
        metrics = []
        for e in range(4):
            eng.train([batch], e)
            metrics.append(eng.test(loader, input_n=10, eval_frame=[1, 5, 10, 29])[1])
        runs.append((eng, metrics))
    (eg, mg), (ee, me) = runs
    assert eg._graph_step is not None and ee._graph_step is None
    for e, (a, b) in enumerate(zip(mg, me)):
        assert np.array_equal(a, b), (e, a, b)
    assert not np.array_equal(mg[0], mg[-1])  # the weights did move between the tests


def test_dropout_mask_is_regenerated_in_backward():
    """do_in dropout (p > 0): the forward mask is a hash of (seed, element),
    so the backward regenerates it; the gradient matches a finite difference
    along a random direction of the input-layer weights."""
    m, d = _model_3dpw()
    m.do_in.p = 0.3
    x = torch.from_numpy(d["train/inp0"]).to(DEV).view(8, 40, 23, 3)
    w = torch.randn(8, 40, 23, 3, device=DEV)
    torch.manual_seed(5)
    y1 = m(x)
    torch.manual_seed(5)
    y2 = m(x)
    assert torch.equal(y1, y2)
    torch.manual_seed(6)
    y3 = m(x)
    assert not torch.equal(y1, y3)
    # gradient w.r.t. the last block's PReLU slope (after do_in) vs finite differences
    p = m.conv_st_out.stgcn[0][0].prelu.weight
    torch.manual_seed(5)
    (m(x) * w).sum().backward()
    gp = float(p.grad)
    eps = 1e-2
    vals = []
    for s in (eps, -eps):
        with torch.no_grad():
            p.add_(s)
        torch.manual_seed(5)
        with torch.no_grad():
            vals.append(float((m(x) * w).sum().double()))
        with torch.no_grad():
            p.sub_(s)
    fd = (vals[0] - vals[1]) / (2 * eps)
    assert abs(fd - gp) <= 2e-2 * max(abs(fd), 1.0), (fd, gp)


# ---- engine: loss and test metric ----------------------------------------------
def test_mpjpe_forward_backward():
    from engine import mpjpe_error_3d
    d = load_npz("engine.npz")
    p = torch.from_numpy(d["mpjpe/pred"]).to(DEV).requires_grad_(True)
    q = torch.from_numpy(d["mpjpe/targ"]).to(DEV)
    v = mpjpe_error_3d(p, q)
    assert abs(float(v) - float(d["mpjpe/value"])) < 1e-5
    (3.0 * v).backward()
    p64 = torch.from_numpy(d["mpjpe/pred"]).double().requires_grad_(True)
    (3.0 * O.mpjpe_error_3d(p64, torch.from_numpy(d["mpjpe/targ"]).double())).backward()
    assert rel(p.grad, p64.grad) < 1e-5


def test_engine_test_metric_matches_reference():
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    d = load_npz("engine.npz")
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=25, st_gcnn_dropout=0.1,
                joints_to_consider=22, num_feature=64, num_layers=5, layout="h36m")
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "test/sd/").items()})
    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    eng = PredictionEngine(cfg, m.to(DEV), _Log())
    inputs = torch.from_numpy(d["test/inputs"])
    all_seqs = torch.from_numpy(d["test/all_seqs"])
    # two batches of 2: per-batch sums accumulate on the device like the reference's t_metric
    loader = [(inputs[:2], None, None, all_seqs[:2]), (inputs[2:], None, None, all_seqs[2:])]
    avg, metric = eng.test(loader, input_n=10, eval_frame=list(d["test/eval_frame"]), dim_used=d["test/dim_used"],
                           joint_to_ignore=d["test/joint_to_ignore"], joint_equal=d["test/joint_equal"])
    ref = d["test/metric"]
    assert np.abs(metric - ref).max() / np.abs(ref).max() < 2e-4
    assert abs(avg - float(d["test/avg"])) / float(d["test/avg"]) < 2e-4


# ---- ST_GCNN_layer(refine=False): ConvTemporalGraphical + KxK conv (§8(f) row 4) ----
PLAIN = {"p_64_32_k31": (64, 32, [3, 1], 35), "p_16_16_k33": (16, 16, [3, 3], 20), "p_8_12_k11": (8, 12, [1, 1], 10)}


@pytest.mark.parametrize("name", list(PLAIN))
def test_plain_st_gcnn_layer_forward_backward(name):
    from model import ST_GCNN_layer
    cin, cout, ks, T = PLAIN[name]
    d = load_npz("plain_layers.npz")
    sd = group(d, f"{name}/sd/")
    layer = ST_GCNN_layer(cin, cout, ks, 1, T, 22, True, False, True, "h36m")
    layer.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    layer = layer.to(DEV)
    x = torch.from_numpy(d[f"{name}/x"])
    xg = x.to(DEV).requires_grad_(True)
    y = layer(xg)
    assert rel(y, torch.from_numpy(d[f"{name}/y64"])) < 1e-4
    w = torch.randn(y.shape)
    (y * w.to(DEV)).sum().backward()
    P = {k: torch.from_numpy(v).double().requires_grad_(not k.endswith("A_fixed")) for k, v in sd.items()}
    x64 = x.double().requires_grad_(True)
    (O.st_gcnn_layer_plain(x64, P, ks, 1) * w.double()).sum().backward()
    assert rel(xg.grad, x64.grad) < 1e-4
    for k, p in layer.named_parameters():
        if k.endswith("A_fixed"):
            assert p.grad is None
            continue
        assert rel(p.grad, P[k].grad) < 1e-4, k


def test_native_conv2d_strided_padded():
    """The KxK Conv2d kernels on a stride-2, asymmetric-padding case."""
    from model import Conv2d
    torch.manual_seed(3)
    conv = Conv2d(5, 7, (3, 5), stride=(2, 1), padding=(1, 2))
    x = torch.randn(2, 5, 11, 9)
    ref = torch.nn.functional.conv2d(x.double(), conv.weight.double(), conv.bias.double(), stride=(2, 1),
                                     padding=(1, 2))
    conv = conv.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    y = conv(xg)
    assert y.shape == ref.shape and rel(y, ref) < 1e-5
    w = torch.randn(ref.shape)
    (y * w.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    W64 = conv.weight.detach().cpu().double().requires_grad_(True)
    b64 = conv.bias.detach().cpu().double().requires_grad_(True)
    (torch.nn.functional.conv2d(x64, W64, b64, stride=(2, 1), padding=(1, 2)) * w.double()).sum().backward()
    assert rel(xg.grad, x64.grad) < 1e-5
    assert rel(conv.weight.grad, W64.grad) < 1e-5
    assert rel(conv.bias.grad, b64.grad) < 1e-5


def test_model_step_gradient_tail_is_propagation():
    """where the whole-model gradient tail comes from.  Every
    DSTDGCB of the fixture step (the engine's paired step) gets the fp64
    oracle step's own block input and upstream gradient (both halves), and
    its native train-mode forward + backward is compared per tensor with fp64
    autograd of the oracle block (scripts/grad_tail_bisect.py prints the
    tables): every parameter and input gradient within the block bar (2e-4,
    test_dstdgcb_train_forward_backward) or within 3x the fp32 oracle's own
    error on the same block over 10 implementations / sample orders -- the
    block's own arithmetic is an fp32 implementation's, so the model-level
    tail is propagation through the ill-conditioned stack, not a kernel's
    summation.  The spatial DSTDGCs of the worst block alone: each op's
    d alpha (a sum cancelling 10^2-10^3-fold) within 2x the fp32 oracle's
    error."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import grad_tail_bisect as GT
    d, batch = GT.batch_np()
    sd0 = group(d, "train/sd0/")
    _, rec = GT.oracle_step(sd0, batch, torch.float64, DEV, record=True)
    worst_b, worst_v = 0, 0.0
    for b in range(len(GT.PREFIXES)):
        pre, rows = GT.block_detail(sd0, rec, b)
        for e, k, sc, tol, ec, eg in rows:
            assert e <= max(1.0, 3.0 * max(ec, eg)), (pre, k, e, ec, eg)
        print(pre, "native err / tol max", round(rows[0][0], 3), rows[0][1])
        if rows[0][0] > worst_v:
            worst_b, worst_v = b, rows[0][0]
    pre, orows = GT.op_detail(sd0, batch, worst_b)
    for i, g64, en, ec, eg, canc in orows:
        assert abs(en) <= 2.0 * max(abs(ec), abs(eg), 1e-6 * abs(g64)), (pre, i, g64, en, ec, eg)
