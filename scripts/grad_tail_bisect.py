"""Where the whole-model gradient tail of the native training step comes from
(VERDICT r04 "what's weak" #1; tests/test_gpu_train.py
test_model_step_gradient_tail_is_propagation holds the same checks as asserts).

On the 3DPW fixture batch (B=8, the engine's paired step: the batch and its
time reversal, engine/prediction.py:231-287):

1. per block: every DSTDGCB of the step gets the fp64 oracle's own block input
   and upstream gradient (both halves of the pair), the native train-mode
   block runs forward + backward on them, and its parameter gradients are
   compared with fp64 autograd of the oracle block on the same inputs
   (model/dstdgcn.py:141-163) -- the block's own arithmetic, nothing inherited;
2. the conditioning of the step: the fp64 step again with every parameter
   moved by one fp32 rounding (relative 2^-24, random signs) -- how far a
   perturbation at fp32 resolution moves each gradient in exact arithmetic;
3. the fp32 noise as a distribution: the fp32 oracle step on the GPU over
   several sample orders of the same batch (the loss and BatchNorm are
   order-invariant, so every order is another fp32 summation order), on the
   CPU, and the reference's own fp32 run.

Prints one table per part."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dstd-gcn_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
from conftest import group, load_npz  # noqa: E402
from oracle import dstdgcn_oracle as O  # noqa: E402

DEV = "cuda:0"
NUM_LAYERS = 5
PREFIXES = (["conv_st_in.stgcn.0.0."] + [f"encoders.{i}.0.stgcn.0.0." for i in range(NUM_LAYERS)] +
            ["conv_st_out.stgcn.0.0."])


def batch_np():
    d = load_npz("engine.npz")
    return d, tuple(d[f"train/{n}0"] for n in ("inp", "inv", "seq"))


def oracle_step(sd0, batch, dtype, dev, perm=None, jitter=None, record=False):
    """The oracle's engine step; returns (grads, per-call block records).
    perm: sample order; jitter: relative parameter perturbation (fp64 only)."""
    P = O.train_params(sd0, dtype, dev)
    if jitter is not None:
        g = torch.Generator().manual_seed(jitter)
        with torch.no_grad():
            for k, v in P.items():
                if v.requires_grad:
                    s = torch.randint(0, 2, v.shape, generator=g).to(v) * 2 - 1
                    v.mul_(1 + s * 2.0 ** -24)
    b = batch if perm is None else tuple(a[perm] for a in batch)
    rec = []
    orig = O.dstdgcb
    if record:
        def hooked(x, p, training=False):
            x_in = x.detach().clone()
            y = orig(x, p, training)
            y.retain_grad()
            rec.append((x_in, y))
            return y
        O.dstdgcb = hooked
    try:
        _, lall = O.step_loss(P, b, NUM_LAYERS)
    finally:
        O.dstdgcb = orig
    lall.backward()
    grads = {k: v.grad.double().cpu().numpy() for k, v in P.items() if v.grad is not None}
    return grads, [(x, y.grad.detach().clone()) for x, y in rec]


def block_detail(sd0, rec, b, n_perm=8):
    """Block b of the step on the fp64 step's own block input and upstream
    gradient (both halves): per parameter gradient (and the input gradient of
    each half, _dx0 / _dx1) (err / tol of the native block, tensor, |ref|,
    tol, err / tol of the fp32 oracle on the CPU, the largest err / tol of the
    fp32 oracle on the GPU over n_perm sample orders -- BatchNorm is
    order-invariant); tol = 2e-4 max(|ref|, 1e-3 x the block's gradient scale)
    as in tests/test_gpu_train.py test_dstdgcb_train_forward_backward."""
    from model import DSTDGCB
    from test_gpu_train import _realias
    nb = len(PREFIXES)
    pre = PREFIXES[b]
    p = O.sub({k: v for k, v in sd0.items()}, pre)
    halves = [rec[b], rec[nb + b]]
    cin, T, V = halves[0][0].shape[1], halves[0][0].shape[2], halves[0][0].shape[3]
    cout = p["conv_s.0.conv_f.weight"].shape[0]

    def oracle(dt, dev, perm=None):
        P = {k: torch.as_tensor(v).to(dev, dt).clone() for k, v in p.items()
             if not k.endswith(("num_batches_tracked", "running_mean", "running_var"))}
        for k in P:
            if not k.endswith(("A_s", "A_t")):
                P[k].requires_grad_(True)
        P["A_s"] = P["R_s"].detach()
        dxs = []
        for x, dy in halves:
            xx = x.detach().to(dev, dt).clone()
            dd = dy.detach().to(dev, dt)
            if perm is not None:
                xx, dd = xx[perm], dd[perm]
            xx.requires_grad_(True)
            y = O.dstdgcb(xx, P, training=True)
            (y * dd).sum().backward()
            g = xx.grad if perm is None else xx.grad[torch.argsort(torch.as_tensor(perm, device=xx.device))]
            dxs.append(g.double().cpu())
        out = {k: v.grad.double().cpu() for k, v in P.items() if v.grad is not None}
        out["_dx0"], out["_dx1"] = dxs
        return out

    r64 = oracle(torch.float64, DEV)
    r32c = oracle(torch.float32, "cpu")
    B = halves[0][0].shape[0]
    r32g = [oracle(torch.float32, DEV, None if s == 0 else np.random.default_rng(s).permutation(B))
            for s in range(n_perm)]
    blk = DSTDGCB(cin, cout, T, V, "3dpw")
    blk.load_state_dict({k: torch.as_tensor(v) for k, v in p.items()})
    blk = blk.to(DEV).train()
    _realias(blk)
    nat = {}
    dxs = []
    for x, dy in halves:
        xg = x.float().to(DEV).requires_grad_(True)
        y = blk(xg)
        (y * dy.float().to(DEV)).sum().backward()
        dxs.append(xg.grad.double().cpu())
    nat = {n: q.grad.double().cpu() for n, q in blk.named_parameters() if q.grad is not None}
    nat["_dx0"], nat["_dx1"] = dxs
    gscale = max(float(v.abs().max()) for k, v in r64.items() if not k.startswith("_"))
    rows = []
    for k, ref in r64.items():
        tol = 2e-4 * max(float(ref.abs().max()), 1e-3 * gscale)
        e = lambda g: float((g[k] - ref).abs().max()) / tol  # noqa: E731
        rows.append((e(nat), k, float(ref.abs().max()), tol, e(r32c), max(e(g) for g in r32g)))
    rows.sort(reverse=True)
    return pre, rows


def op_detail(sd0, batch, b):
    """The spatial DSTDGCs of block b in isolation: each op of the fp64 step
    (both halves) gets its own recorded input, adjacency, alpha and upstream
    gradient; the native op's d alpha against fp64 autograd of the oracle op,
    next to the fp32 oracle's, and the cancellation of d alpha = sum dD E
    (sum |dD E| / |sum dD E|)."""
    from model import DSTDGC
    pre = PREFIXES[b]
    recs = []
    orig_gc, orig_blk = O.dstdgc, O.dstdgcb
    cur = {"blk": None}

    def blk_hook(x, p, training=False):
        cur["blk"] = p
        return orig_blk(x, p, training)

    def gc_hook(x, p, A, alpha, mode):
        if mode == "spatial" and cur["blk"] is not None and cur["blk"].get("_tag") == pre:
            y = orig_gc(x, p, A, alpha, mode)
            y.retain_grad()
            recs.append((x.detach().clone(), {k: v for k, v in p.items()}, A.detach().clone(),
                         alpha.detach().clone(), y))
            return y
        return orig_gc(x, p, A, alpha, mode)

    P = O.train_params(sd0, torch.float64, DEV)
    for k in list(P):
        if k.endswith(".A_s"):
            P[k] = P[k[:-3] + "R_s"].detach()
    orig_sub = O.sub

    def sub_tag(sd, prefix):
        out = orig_sub(sd, prefix)
        if prefix.endswith("stgcn.0.0."):
            out["_tag"] = prefix
        return out

    O.dstdgc, O.dstdgcb, O.sub = gc_hook, blk_hook, sub_tag
    try:
        _, lall = O.step_loss(P, batch, NUM_LAYERS)
    finally:
        O.dstdgc, O.dstdgcb, O.sub = orig_gc, orig_blk, orig_sub
    lall.backward()
    rows = []
    for i, (x, p, A, alpha, y) in enumerate(recs):
        dy = y.grad.detach()
        pw = {k: v.detach() for k, v in p.items() if torch.is_tensor(v)}
        # fp64 / fp32 oracle op gradients w.r.t. alpha on the recorded inputs
        res = {}
        for tag, dt, dev in (("64", torch.float64, DEV), ("32c", torch.float32, "cpu"), ("32g", torch.float32, DEV)):
            q = {k: v.to(dev, dt) for k, v in pw.items()}
            al = alpha.to(dev, dt).clone().requires_grad_(True)
            yy = O.dstdgc(x.to(dev, dt), q, A.to(dev, dt), al, "spatial")
            (yy * dy.to(dev, dt)).sum().backward()
            res[tag] = float(al.grad)
        # cancellation of the sum (fp64)
        with torch.no_grad():
            xf = O.conv1x1(x, pw["conv_f.weight"], pw["conv_f.bias"])
            p1 = O.conv1x1(x, pw["conv_m1.weight"], pw["conv_m1.bias"])
            q1 = O.conv1x1(x, pw["conv_m2.weight"], pw["conv_m2.bias"])
            n, r, t, v = p1.shape
            m = torch.tanh(p1.reshape(n, r * t, v)[:, :, :, None] - q1.reshape(n, r * t, v)[:, :, None, :])
            wrm = pw["conv_rm.weight"].reshape(pw["conv_rm.weight"].shape[0], -1)
            e = torch.einsum("tk,nkvw->ntvw", wrm, m) + pw["conv_rm.bias"].view(1, -1, 1, 1)
            dD = torch.einsum("nctv,nctw->ntvw", xf, dy)
            canc = float((dD * e).abs().sum() / (dD * e).sum().abs())
        # the native op (train mode: exact fp32 training kernels)
        cin, cout = x.shape[1], pw["conv_f.weight"].shape[0]
        op = DSTDGC(cin, cout, x.shape[2], x.shape[3], mode="spatial")
        op.load_state_dict({k: v.float().cpu() for k, v in pw.items() if not k.startswith("_")})
        op = op.to(DEV)
        al = alpha.float().to(DEV).reshape(1).clone().requires_grad_(True)
        yy = op(x.float().to(DEV), A.float().to(DEV), al)
        (yy * dy.float().to(DEV)).sum().backward()
        rows.append((i, res["64"], float(al.grad) - res["64"], res["32c"] - res["64"], res["32g"] - res["64"], canc))
    return pre, rows


def native_step(d, batch):
    """The engine's paired native step (DSTDGCN.forward_pair) on the fixture batch."""
    from engine import mpjpe_error_3d
    from test_gpu_train import _model_3dpw
    m, _ = _model_3dpw()
    inp, inv, seq = (torch.from_numpy(a).to(DEV) for a in batch)
    B, T, VC = inp.shape
    p1, p2 = m.forward_pair(inp.view(B, T, 23, 3), inv.view(B, T, 23, 3))
    loss = mpjpe_error_3d(p1.reshape(B, T, VC), seq)
    ((loss + mpjpe_error_3d(p2.reshape(B, T, VC), seq.flip(1))) / 2).backward()
    return {n: p.grad.double().cpu().numpy() for n, p in m.named_parameters() if p.grad is not None}


def analyse(n_perm=6, n_jitter=3):
    d, batch = batch_np()
    sd0 = group(d, "train/sd0/")
    g64, rec = oracle_step(sd0, batch, torch.float64, DEV, record=True)
    res = {"blocks": [block_detail(sd0, rec, b) for b in range(len(PREFIXES))]}
    worst = max(range(len(PREFIXES)), key=lambda b: res["blocks"][b][1][0][0])
    res["ops"] = op_detail(sd0, batch, worst)
    g = load_npz("train_grads.npz")
    B = batch[0].shape[0]
    noise = {}  # tensor -> list of fp32 errors (several orderings / implementations)
    for k in g64:
        noise[k] = [float(g["g32err/" + k])]
    runs = [("cpu", None), ("gpu", None)] + [("gpu", np.random.default_rng(s).permutation(B)) for s in range(n_perm)]
    for dev, perm in runs:
        gg, _ = oracle_step(sd0, batch, torch.float32, DEV if dev == "gpu" else "cpu", perm=perm)
        for k in g64:
            noise[k].append(float(np.abs(gg[k] - g64[k]).max()))
    jit = {k: [] for k in g64}
    for s in range(n_jitter):
        gj, _ = oracle_step(sd0, batch, torch.float64, DEV, jitter=100 + s)
        for k in g64:
            jit[k].append(float(np.abs(gj[k] - g64[k]).max()))
    nat = native_step(d, batch)
    rows = []
    for k in g64:
        sc = float(np.abs(g64[k]).max())
        err = float(np.abs(nat[k] - g64[k]).max())
        two = max(noise[k][0], noise[k][1], 1e-4 * sc)  # the former two-sample estimate
        dist = max(max(noise[k]), 1e-4 * sc)  # the distribution's max
        rows.append(dict(k=k, scale=sc, err=err, r_two=err / two, r_dist=err / dist,
                         jitter=max(jit[k]), n_med=float(np.median(noise[k])), n_max=max(noise[k]),
                         n_two=two))
    res["rows"] = rows
    return res


def main():
    res = analyse()
    print("per-block bisection (fp64 block inputs + upstream gradients, both halves); err / tol,")
    print("tol = 2e-4 max(|ref|, 1e-3 block gradient scale); fp32 columns: the oracle block, CPU / GPU x 8 orders")
    print(f"{'block':28s} {'native max':>10s} {'tensor':>24s} {'fp32 cpu':>9s} {'fp32 gpu':>9s} "
          f"{'native / max(1, 3 fp32)':>24s}")
    for pre, rows in res["blocks"]:
        e, k, sc, tol, ec, eg = rows[0]
        worst = max(r[0] / max(1.0, 3 * max(r[4], r[5])) for r in rows)
        print(f"{pre:28s} {e:10.3f} {k:>24s} {ec:9.3f} {eg:9.3f} {worst:24.3f}")
    pre, drows = max(res["blocks"], key=lambda x: x[1][0][0])
    print(f"\n{pre}: per tensor")
    print(f"{'tensor':40s} {'|ref|':>10s} {'tol':>10s} {'native':>8s} {'fp32 cpu':>8s} {'fp32 gpu x8 orders':>18s}")
    for e, k, sc, tol, ec, eg in drows[:10]:
        print(f"{k:40s} {sc:10.3g} {tol:10.3g} {e:8.3f} {ec:8.3f} {eg:18.3f}")
    pre, orows = res["ops"]
    print(f"\n{pre}: its spatial DSTDGCs alone (recorded fp64 input / adjacency / alpha / upstream gradient)")
    print(f"{'call':>4s} {'d alpha (fp64)':>15s} {'native err':>11s} {'fp32 cpu err':>12s} {'fp32 gpu err':>12s} "
          f"{'sum|dD E|/|sum dD E|':>21s}")
    for i, g64, en, ec, eg, canc in orows:
        print(f"{i:4d} {g64:15.6g} {en:11.3g} {ec:12.3g} {eg:12.3g} {canc:21.1f}")
    rows = sorted(res["rows"], key=lambda r: -r["r_two"])
    r2 = np.array([r["r_two"] for r in rows])
    rd = np.array([r["r_dist"] for r in rows])
    print(f"\nnative step err / noise: two-sample estimate median {np.median(r2):.2f} p90 {np.quantile(r2, 0.9):.2f} "
          f"max {r2.max():.2f};  distribution max: median {np.median(rd):.2f} p90 {np.quantile(rd, 0.9):.2f} "
          f"max {rd.max():.2f}")
    print(f"{'tensor':58s} {'err':>9s} {'noise2':>9s} {'noise med':>9s} {'noise max':>9s} {'fp64 jit':>9s} "
          f"{'r_two':>6s} {'r_dist':>6s}")
    for r in rows[:16]:
        print(f"{r['k']:58s} {r['err']:9.3g} {r['n_two']:9.3g} {r['n_med']:9.3g} {r['n_max']:9.3g} "
              f"{r['jitter']:9.3g} {r['r_two']:6.2f} {r['r_dist']:6.2f}")


if __name__ == "__main__":
    main()
