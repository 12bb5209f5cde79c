"""CPU oracle for the DSTDGC hot path -- TEST INFRASTRUCTURE ONLY.

A functional restatement of the reference forward (``/root/reference/model/
dstdgcn.py``) written against a plain ``{name: array}`` state dict, in torch on
the CPU, in fp64 (default) or fp32.  It exists to *check* the MI355X path and to
give ``bench.py`` its ``cpu_baseline`` leg; the product never imports it
(only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s baseline may).

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks this restatement
against fixtures produced by running the reference itself in the build
container (``tests/golden/make_golden.py``): per op, per block and whole model
for the h36m / cmu / 3dpw / h36m-T75 configs.

Every function cites the reference lines it restates.
"""
import torch

BN_EPS = 1e-5  # nn.BatchNorm1d default, model/dstdgcn.py:42

# When a list, every train-mode batchnorm() call appends (batch mean, unbiased
# batch variance) in call order -- what nn.BatchNorm1d folds into its running
# statistics (tests compare the native running-stat updates against it).
BN_RECORD = None


def _t(a, dtype, device="cpu"):
    if torch.is_tensor(a):
        return a.detach().to(device, dtype)
    return torch.as_tensor(a, dtype=dtype, device=device)


def conv1x1(x, w, b):
    """nn.Conv2d(cin, cout, 1) on NCTV (model/dstdgcn.py:66-71)."""
    y = torch.einsum("oc,nctv->notv", w.reshape(w.shape[0], w.shape[1]), x)
    return y + b.view(1, -1, 1, 1)


def dstdgc(x, p, A, alpha, mode):
    """DSTDGC.forward (model/dstdgcn.py:80-94).

    x: [N, Cin, T, V]; p: dict with conv_{f,m1,m2,rm}.{weight,bias};
    A: [1, V, V] (spatial) or [1, T, T] (temporal); alpha: scalar tensor.
    """
    xf = conv1x1(x, p["conv_f.weight"], p["conv_f.bias"])            # :81
    p1 = conv1x1(x, p["conv_m1.weight"], p["conv_m1.bias"])          # :82
    q1 = conv1x1(x, p["conv_m2.weight"], p["conv_m2.bias"])
    n, r, t, v = p1.shape
    wrm = p["conv_rm.weight"].reshape(p["conv_rm.weight"].shape[0], -1)
    brm = p["conv_rm.bias"]
    if mode == "spatial":                                             # :83-87
        pk = p1.reshape(n, r * t, v)                                  # k = r*T + t'
        qk = q1.reshape(n, r * t, v)
        m = torch.tanh(pk[:, :, :, None] - qk[:, :, None, :])         # [n, 2T, V, V]
        d = torch.einsum("tk,nkvw->ntvw", wrm, m) + brm.view(1, -1, 1, 1)
        adj = d * alpha + A                                           # [n, T, V, V]
        return torch.einsum("nctv,ntvw->nctw", xf, adj)
    if mode == "temporal":                                            # :88-93
        pk = p1.permute(0, 1, 3, 2).reshape(n, r * v, t)              # k = r*V + v'
        qk = q1.permute(0, 1, 3, 2).reshape(n, r * v, t)
        m = torch.tanh(pk[:, :, :, None] - qk[:, :, None, :])         # [n, 2V, T, T]
        d = torch.einsum("vk,nktu->nvtu", wrm, m) + brm.view(1, -1, 1, 1)
        adj = d * alpha + A                                           # [n, V, T, T]
        return torch.einsum("nctv,nvtu->ncuv", xf, adj)
    raise ValueError(mode)


def batchnorm(x, p, training=False, eps=BN_EPS):
    """BatchNorm wrapper (model/dstdgcn.py:35-50): BN1d over channel c*V+v,
    statistics over (n, t).  Eval uses running stats; train uses batch stats
    (biased variance for normalisation)."""
    n, c, t, v = x.shape
    xc = x.permute(0, 1, 3, 2).reshape(n, c * v, t)
    if training:
        mean = xc.mean(dim=(0, 2))
        var = xc.var(dim=(0, 2), unbiased=False)
        if BN_RECORD is not None:
            BN_RECORD.append((mean.detach().clone(), xc.var(dim=(0, 2), unbiased=True).detach().clone()))
    else:
        mean, var = p["running_mean"], p["running_var"]
    y = (xc - mean.view(1, -1, 1)) / torch.sqrt(var.view(1, -1, 1) + eps)
    y = y * p["weight"].view(1, -1, 1) + p["bias"].view(1, -1, 1)
    return y.reshape(n, c, v, t).permute(0, 1, 3, 2)


def prelu(x, w):
    """nn.PReLU with a single slope (model/dstdgcn.py:132, 284, 291)."""
    return torch.where(x >= 0, x, w.reshape(()) * x)


def sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def dstdgcb(x, p, training=False):
    """DSTDGCB.forward (model/dstdgcn.py:141-163).  ``p`` holds the block's
    state-dict entries without prefix.  R_s aliases A_s in the reference
    (:107-109); the formula below uses whatever the dict holds for both."""
    cin = x.shape[1]
    cout = p["conv_s.0.conv_f.weight"].shape[0]
    if cin != cout:                                                   # :117-121
        r = conv1x1(x, p["residual.0.weight"], p["residual.0.bias"])
        r = batchnorm(r, sub(p, "residual.1.bn."), training)
    else:
        r = x
    y = None
    for i in range(p["A_s"].shape[0]):                                # :145-150
        a = p["A_s"][i:i + 1] * p["W_s"][i:i + 1] + p["R_s"][i:i + 1]
        z = dstdgc(x, sub(p, f"conv_s.{i}."), a, p["alpha_sm"], "spatial")
        y = z if y is None else y + z
    h = prelu(batchnorm(y, sub(p, "bn.bn."), training) + r, p["prelu.weight"])   # :151-154
    a_t = p["A_t"][0:1] + p["R_t"][0:1]                               # :157-162
    return dstdgc(h, sub(p, "conv_t.0."), a_t, p["alpha_tm"], "temporal")


def dstdgcn(x, sd, num_layers, dtype=torch.float64, training=False, device="cpu"):
    """DSTDGCN.forward (model/dstdgcn.py:293-317), dropout treated as eval.

    x: [N, T, V, 3]; sd: reference state dict (numpy or tensors).  ``device``
    other than the CPU only serves scripts/parity_report.py (the reference
    forward's own fp32 error on the GPU box, torch-ROCm ops)."""
    sd = {k: _t(v, dtype, device) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    return dstdgcn_fn(_t(x, dtype, device), sd, num_layers, training)


def dstdgcn_fn(x, sd, num_layers, training=False):
    """dstdgcn() on tensors used as given (autograd flows through them)."""
    residual = x[:, -1:]                                              # :299
    h = torch.cat((x, x - residual), dim=-1).permute(0, 3, 1, 2)      # :298-303
    h = dstdgcb(h, sub(sd, "conv_st_in.stgcn.0.0."), training)        # :305 (residual=None)
    h = prelu(batchnorm(h, sub(sd, "bn_in.bn."), training), sd["prelu.weight"])   # :306-308
    for i in range(num_layers):                                       # :310-311, 278-285
        e = f"encoders.{i}."
        y = dstdgcb(h, sub(sd, e + "0.stgcn.0.0."), training) + h     # Identity residual :247-248
        h = prelu(batchnorm(y, sub(sd, e + "1.bn."), training), sd[e + "2.weight"])
    y = dstdgcb(h, sub(sd, "conv_st_out.stgcn.0.0."), training)       # :313
    return y.permute(0, 2, 3, 1) + residual                           # :314-315


def ctg(x, p):
    """ConvTemporalGraphical.forward (model/dstdgcn.py:185-188)."""
    x = torch.einsum("nctv,vtq->ncqv", x, p["T"])
    return torch.einsum("nctv,tvw->nctw", x, p["A"] + p["A_fixed"])


def st_gcnn_layer_plain(x, p, kernel_size, stride):
    """ST_GCNN_layer(refine=False).forward (model/dstdgcn.py:218-223, 234-249):
    ConvTemporalGraphical, then Conv2d(kernel_size, stride, 'same' padding),
    plus the residual (Conv2d 1x1 when present in ``p``, else identity)."""
    pad = ((kernel_size[0] - 1) // 2, (kernel_size[1] - 1) // 2)
    y = ctg(x, sub(p, "stgcn.0."))
    y = torch.nn.functional.conv2d(y, p["stgcn.1.weight"], p["stgcn.1.bias"], stride=stride, padding=pad)
    if "residual.weight" in p:
        return y + torch.nn.functional.conv2d(x, p["residual.weight"], p["residual.bias"])
    return y + x


def dstdgcb_forward(x, sd, dtype=torch.float64):
    sd = {k: _t(v, dtype) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    return dstdgcb(_t(x, dtype), sd)


def dstdgc_forward(x, sd, A, alpha, mode, dtype=torch.float64):
    sd = {k: _t(v, dtype) for k, v in sd.items()}
    return dstdgc(_t(x, dtype), sd, _t(A, dtype), _t(alpha, dtype).reshape(()), mode)


# ---------------------------------------------------------------------------
# model/dstdgcn_fast.py: the channels-last variant.  Activations are NTVC,
# conv_f and the block residual are nn.Linear, the spatial adjacency is the
# trainable A_s itself, BN channels are ordered (v, c), and the graph product
# contracts the adjacency's second index (matmul(xm, xf)).
# ---------------------------------------------------------------------------
def fast_dstdgc(x, p, A, alpha, mode):
    """dstdgcn_fast.DSTDGC.forward (model/dstdgcn_fast.py:108-155).

    x: [N, T, V, Cin] -> [N, T, V, Cout]; A: [1, V, V] / [1, T, T]."""
    wf, bf = p["conv_f.weight"], p["conv_f.bias"]                     # nn.Linear :95
    wrm = p["conv_rm.weight"].reshape(p["conv_rm.weight"].shape[0], -1)
    brm = p["conv_rm.bias"]
    if mode == "spatial":                                             # :111-125
        xf = x @ wf.t() + bf                                          # [n, t, v, co]
        xp = x.permute(0, 3, 1, 2)                                    # [n, c, t, v]
        p1 = conv1x1(xp, p["conv_m1.weight"], p["conv_m1.bias"])
        q1 = conv1x1(xp, p["conv_m2.weight"], p["conv_m2.bias"])
        n, r, t, v = p1.shape
        m = torch.tanh(p1.reshape(n, r * t, v)[:, :, :, None] - q1.reshape(n, r * t, v)[:, :, None, :])
        adj = (torch.einsum("tk,nkvw->ntvw", wrm, m) + brm.view(1, -1, 1, 1)) * alpha + A
        return torch.einsum("ntvw,ntwc->ntvc", adj, xf)               # matmul(xm, xf) :125
    if mode == "temporal":                                            # :133-146
        xp = x.permute(0, 3, 2, 1)                                    # [n, c, v, t]
        xf = x.permute(0, 2, 1, 3) @ wf.t() + bf                      # [n, v, t, co]
        p1 = conv1x1(xp, p["conv_m1.weight"], p["conv_m1.bias"])      # [n, 2, v, t]
        q1 = conv1x1(xp, p["conv_m2.weight"], p["conv_m2.bias"])
        n, r, v, t = p1.shape
        m = torch.tanh(p1.reshape(n, r * v, t)[:, :, :, None] - q1.reshape(n, r * v, t)[:, :, None, :])
        adj = (torch.einsum("vk,nktu->nvtu", wrm, m) + brm.view(1, -1, 1, 1)) * alpha + A
        return torch.einsum("nvtu,nvuc->nvtc", adj, xf).permute(0, 2, 1, 3)   # :145-146
    raise ValueError(mode)


def fast_batchnorm(x, p, training=False, eps=BN_EPS):
    """dstdgcn_fast.BatchNorm (model/dstdgcn_fast.py:41-56): BN1d over channel
    v*C + c of an NTVC tensor, statistics over (n, t)."""
    n, t, v, c = x.shape
    xc = x.permute(0, 2, 3, 1).reshape(n, v * c, t)
    if training:
        mean = xc.mean(dim=(0, 2))
        var = xc.var(dim=(0, 2), unbiased=False)
        if BN_RECORD is not None:
            BN_RECORD.append((mean.detach().clone(), xc.var(dim=(0, 2), unbiased=True).detach().clone()))
    else:
        mean, var = p["running_mean"], p["running_var"]
    y = (xc - mean.view(1, -1, 1)) / torch.sqrt(var.view(1, -1, 1) + eps)
    y = y * p["weight"].view(1, -1, 1) + p["bias"].view(1, -1, 1)
    return y.reshape(n, v, c, t).permute(0, 3, 1, 2)


def fast_dstdgcb(x, p, training=False):
    """dstdgcn_fast.DSTDGCB.forward (model/dstdgcn_fast.py:248-275)."""
    cin = x.shape[-1]
    cout = p["conv_s.0.conv_f.weight"].shape[0]
    if cin != cout:                                                   # :183-188 Linear + BN
        r = x @ p["residual.0.weight"].t() + p["residual.0.bias"]
        r = fast_batchnorm(r, sub(p, "residual.1.bn."), training)
    else:
        r = x
    y = None
    for i in range(p["A_s"].shape[0]):                                # :255-258 (A_s itself)
        z = fast_dstdgc(x, sub(p, f"conv_s.{i}."), p["A_s"][i:i + 1], p["alpha_sm"], "spatial")
        y = z if y is None else y + z
    h = prelu(fast_batchnorm(y, sub(p, "bn.bn."), training) + r, p["prelu.weight"])   # :259-262
    a_t = p["A_t"][0:1] + p["R_t"][0:1]                               # :266-271
    return fast_dstdgc(h, sub(p, "conv_t.0."), a_t, p["alpha_tm"], "temporal")


def fast_dstdgcn_fn(x, sd, num_layers, training=False):
    """dstdgcn_fast.DSTDGCN.forward (model/dstdgcn_fast.py:548-614) on
    tensors used as given; dropout treated as eval."""
    residual = x[:, -1:]                                              # :555
    h = torch.cat((x, x - residual), dim=-1)                          # :558-559 (stays NTVC)
    h = fast_dstdgcb(h, sub(sd, "conv_st_in.stgcn.0.0."), training)   # :563
    h = prelu(fast_batchnorm(h, sub(sd, "bn_in.bn."), training), sd["prelu.weight"])   # :570-572
    for i in range(num_layers):                                       # :583-584
        e = f"encoders.{i}."
        y = fast_dstdgcb(h, sub(sd, e + "0.stgcn.0.0."), training) + h
        h = prelu(fast_batchnorm(y, sub(sd, e + "1.bn."), training), sd[e + "2.weight"])
    y = fast_dstdgcb(h, sub(sd, "conv_st_out.stgcn.0.0."), training)  # :601
    return y + residual                                               # :610


def fast_dstdgcn(x, sd, num_layers, dtype=torch.float64, training=False):
    sd = {k: _t(v, dtype) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    return fast_dstdgcn_fn(_t(x, dtype), sd, num_layers, training)


def fast_dstdgcb_forward(x, sd, dtype=torch.float64):
    sd = {k: _t(v, dtype) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    return fast_dstdgcb(_t(x, dtype), sd)


def fast_dstdgc_forward(x, sd, A, alpha, mode, dtype=torch.float64):
    sd = {k: _t(v, dtype) for k, v in sd.items()}
    return fast_dstdgc(_t(x, dtype), sd, _t(A, dtype), _t(alpha, dtype).reshape(()), mode)


def mpjpe_error_3d(outputs, targets):
    """engine/utils/loss.py:52-65 with joint_weights=None (all-ones weights:
    the broadcast makes it a plain mean of per-joint L2)."""
    n, t, vc = outputs.shape
    d = (outputs.reshape(-1, 3) - targets.reshape(-1, 3)).norm(dim=1)
    return d.mean()


# ---------------------------------------------------------------------------
# engine restatements (engine/prediction.py, engine/utils/loss.py)
# ---------------------------------------------------------------------------
def test_metric(all_seqs, outputs, input_n, eval_frame, dim_used, joint_to_ignore, joint_equal):
    """PredictionEngine.test per-frame MPJPE for one batch (prediction.py:366-404),
    numpy.  Returns (metric_k * n for each k) as the reference accumulates it."""
    import numpy as np
    all_seqs = np.asarray(all_seqs, dtype=np.float64)
    outputs = np.asarray(outputs, dtype=np.float64)
    n, seq_len, D = all_seqs.shape
    pred = all_seqs.copy()
    if outputs.shape[1] != seq_len:                                   # :371-381
        pred[:, input_n:, dim_used] = outputs
    else:
        pred[:, :, dim_used] = outputs
    ign = np.concatenate((joint_to_ignore * 3, joint_to_ignore * 3 + 1, joint_to_ignore * 3 + 2))
    eq = np.concatenate((joint_equal * 3, joint_equal * 3 + 1, joint_equal * 3 + 2))
    pred[:, :, ign] = pred[:, :, eq]                                  # :382-389
    p = pred.reshape(n, seq_len, -1, 3)[:, input_n:]
    t = all_seqs.reshape(n, seq_len, -1, 3)[:, input_n:]
    return np.array([np.linalg.norm(t[:, j] - p[:, j], axis=-1).mean() * n for j in eval_frame])


def train_params(sd0, dtype=torch.float64, device="cpu"):
    """Leaf tensors for training: every state-dict parameter except A_s / A_t
    requires grad; BN running statistics are dropped (train-mode BN never
    reads them).  ``device`` other than the CPU: the same torch ops on the GPU
    box's torch-ROCm (tests at training batches, where the CPU takes a minute)."""
    P = {k: _t(v, dtype, device).clone() for k, v in sd0.items()
         if not k.endswith(("num_batches_tracked", "running_mean", "running_var"))}
    for k in P:
        if not k.endswith((".A_s", ".A_t")):
            P[k].requires_grad_(True)
    return P


def step_loss(P, batch, num_layers, inverse=True):
    """Losses of one PredictionEngine.train step (prediction.py:231-287):
    returns (loss, all_loss) with all_loss = (loss + loss_inv) / 2 when
    ``inverse``.  A_s re-reads R_s's values (the storage alias, :107-109)."""
    p0 = next(iter(P.values()))
    inp, inv, seq = (_t(a, p0.dtype, p0.device) for a in batch)
    B, T, VC = inp.shape
    for k in list(P):
        if k.endswith(".A_s"):
            P[k] = P[k[:-3] + "R_s"].detach()
    out = dstdgcn_fn(inp.view(B, T, VC // 3, 3), P, num_layers, training=True).reshape(B, T, VC)
    loss = mpjpe_error_3d(out, seq)
    if not inverse:
        return loss, loss
    out_i = dstdgcn_fn(inv.view(B, T, VC // 3, 3), P, num_layers, training=True).reshape(B, T, VC)
    return loss, (loss + mpjpe_error_3d(out_i, seq.flip(1))) / 2


def train_curve(sd0, batches, steps, num_layers, lr=3e-3, weight_decay=0.0, inverse=True, dtype=torch.float64):
    """PredictionEngine.train for ``steps`` one-batch epochs (prediction.py:198-317):
    train-mode forward, mpjpe loss, the time-reversed pass, all_loss / 2,
    Adam(lr, weight_decay).  ``batches``: list of (inputs, inputs_inv,
    targets) as [B, T, V*3] arrays.  Returns the per-step loss of the forward
    pass (the t_l average the engine reports)."""
    P = train_params(sd0, dtype)
    opt = torch.optim.Adam([v for v in P.values() if v.requires_grad], lr=lr, weight_decay=weight_decay)
    losses = []
    for step in range(steps):
        loss, all_loss = step_loss(P, batches[step % len(batches)], num_layers, inverse)
        opt.zero_grad()
        all_loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    return losses
