#!/usr/bin/env python
"""Generate the golden parity fixtures by running the REFERENCE implementation.

This script is the only place that executes reference code, and it runs only in
the build container (``/root/reference`` does not exist on the GPU box).  It
imports ``model/`` and ``engine/`` from the reference checkout, builds the ops,
blocks and whole models named in SURVEY.md §8(c), randomises the parameters that
are zero at init (``alpha_sm``, ``alpha_tm``, ``W_s``, ``R_t`` -- SURVEY §0.6),
calibrates BatchNorm running statistics with train-mode passes, and records the
inputs, the full ``state_dict`` and the outputs in fp32 and fp64 as ``.npz``
files next to this script.  Nothing is pickled: every array is plain numpy.

Usage:  python tests/golden/make_golden.py            (writes tests/golden/*.npz)

Fixture list (all committed):
  graphs.npz          Graph(layout).get_all_adjacency(), Time(T).get_all_adjacency()
  dstdgc_ops.npz      single DSTDGC ops (spatial/temporal), random A, random alpha
  dstdgcb.npz         DSTDGCB blocks 64->64, 6->64, 64->3 with calibrated BN
  model_<cfg>.npz     whole DSTDGCN (h36m, cmu, 3dpw, h36m75) at B=4
  engine.npz          mpjpe_error_3d + PredictionEngine.test metric + 3DPW loss curve
  train_grads.npz     fp64 gradients / loss curve of the engine.npz training run
  plain_layers.npz    ST_GCNN_layer(refine=False): ConvTemporalGraphical + KxK conv
  dstdgcn_fast.npz    model/dstdgcn_fast.py (channels-last variant): ops, blocks,
                      whole models (h36m, 3dpw) and fp64 gradients of one step

``python tests/golden/make_golden.py train`` / ``plain`` / ``fast`` regenerates
train_grads.npz / plain_layers.npz / dstdgcn_fast.npz only.
"""
import copy
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from model import get_model  # noqa: E402  (reference)
from model.dstdgcn import DSTDGC, DSTDGCB  # noqa: E402  (reference)
from model.layers.graph import Graph  # noqa: E402  (reference)
from model.layers.time import Time  # noqa: E402  (reference)

# shapes per BASELINE.json / SURVEY §0.3
CONFIGS = {
    "h36m": dict(layout="h36m", V=22, Tin=10, Tout=25),
    "cmu": dict(layout="cmu", V=25, Tin=10, Tout=25),
    "3dpw": dict(layout="3dpw", V=23, Tin=10, Tout=30),
    "h36m75": dict(layout="h36m", V=22, Tin=50, Tout=25),
}


def synth_input(gen, B, T, V, Tin, C=3):
    """N(0,1) poses; future frames padded with the last observed one
    (dataset/h36m.py:53-64 convention)."""
    x = torch.randn(B, T, V, C, generator=gen, dtype=torch.float32)
    x[:, Tin:] = x[:, Tin - 1:Tin]
    return x


def randomise_dynamic(block, gen):
    """Make the dynamic terms of a DSTDGCB non-trivial."""
    with torch.no_grad():
        block.alpha_sm.copy_(torch.empty(1).uniform_(0.3, 1.0, generator=gen) *
                             (1 if torch.rand(1, generator=gen) > 0.3 else -1))
        block.alpha_tm.copy_(torch.empty(1).uniform_(0.3, 1.0, generator=gen))
        block.W_s.copy_(0.3 * torch.randn(block.W_s.shape, generator=gen))
        # R_s aliases A_s (model/dstdgcn.py:107-109): perturbing it moves both
        block.R_s.add_(0.1 * torch.randn(block.R_s.shape, generator=gen))
        T = block.R_t.shape[-1]
        block.R_t.copy_(torch.empty(block.R_t.shape).uniform_(-1 / T**0.5, 1 / T**0.5, generator=gen))
        block.prelu.weight.copy_(torch.empty(1).uniform_(0.1, 0.4, generator=gen))


def perturb_bn(module, gen):
    with torch.no_grad():
        for m in module.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.weight.copy_(torch.empty(m.weight.shape).uniform_(0.8, 1.2, generator=gen))
                m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=gen))
            if isinstance(m, torch.nn.PReLU):
                m.weight.copy_(torch.empty(1).uniform_(0.1, 0.4, generator=gen))


def calibrate(module, make_x, passes=20):
    module.train()
    with torch.no_grad():
        for _ in range(passes):
            module(make_x())
    module.eval()


def sd_numpy(module, prefix=""):
    out = {}
    for k, v in module.state_dict().items():
        out[prefix + k] = v.detach().cpu().numpy().copy()
    return out


def run64(module, *args):
    m64 = copy.deepcopy(module).double().eval()
    with torch.no_grad():
        return m64(*[a.double() if torch.is_tensor(a) else a for a in args]).numpy()


def put_outputs(out, prefix, y32, y64):
    """Store the fp64 reference output rounded to fp32 (6e-8 relative, far
    below the 1e-4 parity bar) plus the reference's own fp32-vs-fp64 error
     so tests can scale tolerances without storing y32."""
    out[prefix + "y64"] = y64.astype(np.float32)
    out[prefix + "ref32_err"] = np.array(np.abs(y32 - y64).max() / np.abs(y64).max())


def gen_graphs():
    out = {}
    for layout in ("h36m", "cmu", "3dpw"):
        out[f"graph_{layout}"] = Graph(layout).get_all_adjacency()
    for T in (6, 35, 40, 75):
        out[f"time_{T}"] = Time(T).get_all_adjacency()
    np.savez_compressed(os.path.join(HERE, "graphs.npz"), **out)


def gen_ops(gen):
    cases = [
        # name, mode, cin, cout, T, V
        ("s_64_64_h36m", "spatial", 64, 64, 35, 22),
        ("s_6_64_h36m", "spatial", 6, 64, 35, 22),
        ("s_64_3_h36m", "spatial", 64, 3, 35, 22),
        ("s_64_64_cmu", "spatial", 64, 64, 35, 25),
        ("t_64_64_h36m", "temporal", 64, 64, 35, 22),
        ("t_3_3_h36m", "temporal", 3, 3, 35, 22),
        ("t_64_64_3dpw", "temporal", 64, 64, 40, 23),
        ("t_64_64_h36m75", "temporal", 64, 64, 75, 22),
    ]
    out = {}
    B = 1
    for name, mode, cin, cout, T, V in cases:
        ref, kpt = (T, V) if mode == "spatial" else (V, T)
        op = DSTDGC(cin, cout, ref, kpt, mode=mode).eval()
        with torch.no_grad():
            for p in op.parameters():  # biases are 0 at init: make them matter
                if p.dim() == 1:
                    p.copy_(0.1 * torch.randn(p.shape, generator=gen))
        Ad = V if mode == "spatial" else T
        A = torch.randn(1, Ad, Ad, generator=gen) * 0.3
        alpha = torch.empty(1).uniform_(0.5, 1.5, generator=gen)
        x = torch.randn(B, cin, T, V, generator=gen)
        with torch.no_grad():
            y32 = op(x, A, alpha).numpy()
        y64 = run64(op, x, A, alpha)
        out[f"{name}/x"] = x.numpy()
        out[f"{name}/A"] = A.numpy()
        out[f"{name}/alpha"] = alpha.numpy()
        put_outputs(out, f"{name}/", y32, y64)
        for k, v in sd_numpy(op).items():
            out[f"{name}/sd/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "dstdgc_ops.npz"), **out)


def gen_blocks(gen):
    cases = [("b_64_64_h36m", 64, 64, "h36m", 35, 22), ("b_6_64_h36m", 6, 64, "h36m", 35, 22),
             ("b_64_3_h36m", 64, 3, "h36m", 35, 22), ("b_64_64_cmu", 64, 64, "cmu", 35, 25)]
    out = {}
    B = 1
    for name, cin, cout, layout, T, V in cases:
        blk = DSTDGCB(cin, cout, T, V, layout)
        randomise_dynamic(blk, gen)
        perturb_bn(blk, gen)
        with torch.no_grad():
            for m in blk.modules():
                if isinstance(m, torch.nn.Conv2d):
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=gen))
        calibrate(blk, lambda: torch.randn(8, cin, T, V, generator=gen))
        x = torch.randn(B, cin, T, V, generator=gen)
        with torch.no_grad():
            y32 = blk(x).numpy()
        y64 = run64(blk, x)
        out[f"{name}/x"] = x.numpy()
        put_outputs(out, f"{name}/", y32, y64)
        for k, v in sd_numpy(blk).items():
            out[f"{name}/sd/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "dstdgcb.npz"), **out)


def build_model(cfg, gen, dropout=0.1):
    opts = dict(input_channels=6, input_time_frame=cfg["Tin"], output_time_frame=cfg["Tout"],
                st_gcnn_dropout=dropout, joints_to_consider=cfg["V"], num_feature=64, num_layers=5,
                layout=cfg["layout"])
    model = get_model("dstdgcn", dstdgcn=opts)
    for m in model.modules():
        if isinstance(m, DSTDGCB):
            randomise_dynamic(m, gen)
    perturb_bn(model, gen)
    return model, opts


def gen_models(gen):
    for tag, cfg in CONFIGS.items():
        model, opts = build_model(cfg, gen)
        T = cfg["Tin"] + cfg["Tout"]
        calibrate(model, lambda: synth_input(gen, 16, T, cfg["V"], cfg["Tin"]))
        x = synth_input(gen, 4, T, cfg["V"], cfg["Tin"])
        with torch.no_grad():
            y32 = model(x).numpy()
        y64 = run64(model, x)
        out = {"x": x.numpy()}
        put_outputs(out, "", y32, y64)
        for k, v in opts.items():
            out[f"opt/{k}"] = np.array(v)
        for k, v in sd_numpy(model).items():
            out[f"sd/{k}"] = v
        np.savez_compressed(os.path.join(HERE, f"model_{tag}.npz"), **out)


def gen_engine(gen):
    """mpjpe_error_3d, the PredictionEngine.test metric and a short 3DPW
    config-5 training curve (engine/prediction.py:198-317, 319-430)."""
    from engine.utils.loss import mpjpe_error_3d  # reference
    from engine.prediction import PredictionEngine  # reference

    out = {}
    pred = torch.randn(3, 7, 22 * 3, generator=gen)
    targ = torch.randn(3, 7, 22 * 3, generator=gen)
    out["mpjpe/pred"] = pred.numpy()
    out["mpjpe/targ"] = targ.numpy()
    out["mpjpe/value"] = np.array(mpjpe_error_3d(pred, targ).item())

    class _Log:
        def info(self, *a, **k):
            pass

    # reference engine moves batches with .cuda(); identity on this CPU-only box
    torch.Tensor.cuda = lambda self, *a, **k: self

    cfg = CONFIGS["h36m"]
    T = cfg["Tin"] + cfg["Tout"]
    model, _ = build_model(cfg, gen)
    calibrate(model, lambda: synth_input(gen, 16, T, cfg["V"], cfg["Tin"]))
    eng_cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
                   loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    engine = PredictionEngine(eng_cfg, model, _Log())
    # one synthetic test batch: 32 H36M joints x 3 = 96 dims, 22 used
    n = 4
    all_seqs = torch.randn(n, T, 96, generator=gen)
    dim_used = np.array([6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,
                         36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 51, 52, 53, 54, 55, 56, 57, 58, 59, 63, 64,
                         65, 66, 67, 68, 75, 76, 77, 78, 79, 80, 81, 82, 83, 87, 88, 89, 90, 91, 92])
    inputs = all_seqs[:, :, dim_used].clone()
    inputs[:, cfg["Tin"]:] = inputs[:, cfg["Tin"] - 1:cfg["Tin"]]
    j_ign = np.array([16, 20, 23, 24, 28, 31])
    j_eq = np.array([13, 19, 22, 13, 27, 30])
    eval_frame = [1, 3, 7, 9, 13, 24]
    loader = [(inputs, None, None, all_seqs)]
    avg, metric = engine.test(loader, input_n=cfg["Tin"], eval_frame=eval_frame, dim_used=dim_used,
                              joint_to_ignore=j_ign, joint_equal=j_eq)
    out["test/all_seqs"] = all_seqs.numpy()
    out["test/inputs"] = inputs.numpy()
    out["test/dim_used"] = dim_used
    out["test/joint_to_ignore"] = j_ign
    out["test/joint_equal"] = j_eq
    out["test/eval_frame"] = np.array(eval_frame)
    out["test/avg"] = np.array(avg)
    out["test/metric"] = metric
    for k, v in sd_numpy(model).items():
        out[f"test/sd/{k}"] = v

    # 3DPW config-5 style loss curve: dropout 0 (dstdgcn_3dpw.yaml:137), inverse=True
    cfg = CONFIGS["3dpw"]
    T = cfg["Tin"] + cfg["Tout"]
    torch.manual_seed(0)
    model, _ = build_model(cfg, gen, dropout=0.0)
    out.update({f"train/sd0/{k}": v for k, v in sd_numpy(model).items()})
    engine = PredictionEngine(eng_cfg, model, _Log())
    batches = []
    for _ in range(4):
        seq = torch.randn(8, T, cfg["V"] * 3, generator=gen)
        inp = seq.clone()
        inp[:, cfg["Tin"]:] = inp[:, cfg["Tin"] - 1:cfg["Tin"]]
        inv = seq.flip(1).clone()
        inv[:, cfg["Tin"]:] = inv[:, cfg["Tin"] - 1:cfg["Tin"]]
        batches.append((inp, inv, seq, seq))
    losses = []
    for step in range(5):
        losses.append(engine.train([batches[step % 4]], step, max_iter=1))
    for i, (inp, inv, seq, _) in enumerate(batches):
        out[f"train/inp{i}"] = inp.numpy()
        out[f"train/inv{i}"] = inv.numpy()
        out[f"train/seq{i}"] = seq.numpy()
    out["train/losses"] = np.array(losses)
    np.savez_compressed(os.path.join(HERE, "engine.npz"), **out)


def _realias(model):
    """.double() copies every parameter separately and so breaks the A_s/R_s
    storage alias (model/dstdgcn.py:107-109); point A_s back at R_s."""
    for m in model.modules():
        if isinstance(m, DSTDGCB):
            m.A_s.data = m.R_s.data


def gen_train_grads(gen):
    """fp64 ground truth for the training path, on the
    engine.npz 3DPW model and batches:
      g64/<param>   gradient of step 0's all_loss = (loss + loss_inv) / 2
                    (engine/prediction.py:258-290) in fp64
      g32err/<param> max |g32 - g64| of the reference's own fp32 gradient
      losses64      the 5-step curve of engine.npz train/losses in fp64
    fp32 training of this model is chaotic (ref fp32 vs fp64 gradients differ
    by up to ~1x on parameters whose true gradient is ~0, e.g. a conv bias in
    front of BatchNorm), so parity is judged against fp64 with the reference's
    own fp32 error as the yardstick."""
    from engine.utils.loss import mpjpe_error_3d  # reference

    d = np.load(os.path.join(HERE, "engine.npz"))
    sd0 = {k[len("train/sd0/"):]: d[k] for k in d.files if k.startswith("train/sd0/")}
    cfg = CONFIGS["3dpw"]
    opts = dict(input_channels=6, input_time_frame=cfg["Tin"], output_time_frame=cfg["Tout"], st_gcnn_dropout=0.0,
                joints_to_consider=cfg["V"], num_feature=64, num_layers=5, layout=cfg["layout"])
    batches = [tuple(torch.from_numpy(d[f"train/{n}{i}"]) for n in ("inp", "inv", "seq")) for i in range(4)]

    def build(dtype):
        m = get_model("dstdgcn", dstdgcn=opts)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd0.items()})
        if dtype == torch.float64:
            m = m.double()
            _realias(m)
        return m.train()

    def grads(dtype):
        m = build(dtype)
        inp, inv, seq = (b.to(dtype) for b in batches[0])
        B, T, VC = inp.shape
        out = m(inp.view(B, T, VC // 3, 3)).reshape(B, T, VC)
        out_i = m(inv.view(B, T, VC // 3, 3)).reshape(B, T, VC)
        loss = (mpjpe_error_3d(out, seq) + mpjpe_error_3d(out_i, seq.flip(1))) / 2
        loss.backward()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    g64, g32 = grads(torch.float64), grads(torch.float32)
    out = {}
    for k in g64:
        out[f"g64/{k}"] = g64[k].numpy()
        out[f"g32err/{k}"] = np.array(float((g32[k].double() - g64[k]).abs().max()))

    def curve(dtype):
        # PredictionEngine.train's step (prediction.py:231-294) on the reference
        # modules; the engine itself casts batches to fp32 (:223-225), so the
        # fp64 curve runs this restatement (checked against the engine's own
        # fp32 curve below).
        m = build(dtype)
        opt = torch.optim.Adam(m.parameters(), lr=3e-3, weight_decay=0)
        losses = []
        for step in range(5):
            inp, inv, seq = (b.to(dtype) for b in batches[step % 4])
            B, T, VC = inp.shape
            loss = mpjpe_error_3d(m(inp.view(B, T, VC // 3, 3)).reshape(B, T, VC), seq)
            loss_i = mpjpe_error_3d(m(inv.view(B, T, VC // 3, 3)).reshape(B, T, VC), seq.flip(1))
            opt.zero_grad()
            ((loss + loss_i) / 2).backward()
            opt.step()
            losses.append(float(loss.item()))
        return np.array(losses)

    c32 = curve(torch.float32)
    assert np.abs(c32 - d["train/losses"]).max() < 1e-5 * d["train/losses"].max(), (c32, d["train/losses"])
    out["losses64"] = curve(torch.float64)
    np.savez_compressed(os.path.join(HERE, "train_grads.npz"), **out)


def gen_plain_layers(gen):
    """ST_GCNN_layer(refine=False): ConvTemporalGraphical + k_t x k_v Conv2d
    (model/dstdgcn.py:166-188, 218-223) -- dead in the shipped configs, kept
    for API completeness."""
    from model.dstdgcn import ST_GCNN_layer  # reference
    cases = [("p_64_32_k31", 64, 32, [3, 1], 1, 35, 22), ("p_16_16_k33", 16, 16, [3, 3], 1, 20, 22),
             ("p_8_12_k11", 8, 12, [1, 1], 1, 10, 22)]
    out = {}
    for name, cin, cout, ks, stride, T, V in cases:
        layer = ST_GCNN_layer(cin, cout, ks, stride, T, V, True, False, True, "h36m")
        with torch.no_grad():
            for m in layer.modules():
                if isinstance(m, torch.nn.Conv2d):
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=gen))
        x = torch.randn(2, cin, T, V, generator=gen)
        with torch.no_grad():
            y32 = layer(x).numpy()
        y64 = run64(layer, x)
        out[f"{name}/x"] = x.numpy()
        put_outputs(out, f"{name}/", y32, y64)
        for k, v in sd_numpy(layer).items():
            out[f"{name}/sd/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "plain_layers.npz"), **out)


def gen_fast(gen):
    """model/dstdgcn_fast.py: the channels-last variant (NTVC activations,
    conv_f / residual as nn.Linear, a trainable A_s without W_s / R_s, BN
    channels ordered (v, c), and the graph product contracted on the other
    adjacency index: matmul(xm, xf), :125 / :145)."""
    from model import dstdgcn_fast as F  # reference
    from engine.utils.loss import mpjpe_error_3d  # reference

    out = {}

    def randomise_fast(block):
        with torch.no_grad():
            block.alpha_sm.copy_(torch.empty(1).uniform_(0.3, 1.0, generator=gen) *
                                 (1 if torch.rand(1, generator=gen) > 0.3 else -1))
            block.alpha_tm.copy_(torch.empty(1).uniform_(0.3, 1.0, generator=gen))
            block.A_s.add_(0.1 * torch.randn(block.A_s.shape, generator=gen))
            T = block.R_t.shape[-1]
            block.R_t.copy_(torch.empty(block.R_t.shape).uniform_(-1 / T**0.5, 1 / T**0.5, generator=gen))
            block.prelu.weight.copy_(torch.empty(1).uniform_(0.1, 0.4, generator=gen))

    def bias_noise(module):
        with torch.no_grad():
            for m in module.modules():
                if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)) and m.bias is not None:
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=gen))

    # single ops: x [B][T][V][C] -> y [B][T][V][Cout]
    for name, mode, cin, cout, T, V in (("op_s_64_64", "spatial", 64, 64, 35, 22),
                                        ("op_s_6_64", "spatial", 6, 64, 35, 22),
                                        ("op_t_64_64", "temporal", 64, 64, 35, 22),
                                        ("op_t_64_64_3dpw", "temporal", 64, 64, 40, 23)):
        ref, kpt = (T, V) if mode == "spatial" else (V, T)
        op = F.DSTDGC(cin, cout, ref, kpt, mode=mode).eval()
        bias_noise(op)
        Ad = V if mode == "spatial" else T
        A = torch.randn(1, Ad, Ad, generator=gen) * 0.3
        alpha = torch.empty(1).uniform_(0.5, 1.5, generator=gen)
        x = torch.randn(1, T, V, cin, generator=gen)
        with torch.no_grad():
            y32 = op(x, A, alpha).numpy()
        y64 = run64(op, x, A, alpha)
        out.update({f"{name}/x": x.numpy(), f"{name}/A": A.numpy(), f"{name}/alpha": alpha.numpy()})
        put_outputs(out, f"{name}/", y32, y64)
        out.update({f"{name}/sd/{k}": v for k, v in sd_numpy(op).items()})

    # blocks (eval, calibrated BN)
    for name, cin, cout, layout, T, V in (("blk_64_64", 64, 64, "h36m", 35, 22), ("blk_6_64", 6, 64, "h36m", 35, 22),
                                          ("blk_64_3", 64, 3, "h36m", 35, 22), ("blk_64_64_cmu", 64, 64, "cmu", 35, 25)):
        blk = F.DSTDGCB(cin, cout, T, V, layout)
        randomise_fast(blk)
        perturb_bn(blk, gen)
        bias_noise(blk)
        calibrate(blk, lambda: torch.randn(8, T, V, cin, generator=gen))
        x = torch.randn(1, T, V, cin, generator=gen)
        with torch.no_grad():
            y32 = blk(x).numpy()
        y64 = run64(blk, x)
        out[f"{name}/x"] = x.numpy()
        put_outputs(out, f"{name}/", y32, y64)
        out.update({f"{name}/sd/{k}": v for k, v in sd_numpy(blk).items()})

    def build(cfg, dropout):
        opts = dict(input_channels=6, input_time_frame=cfg["Tin"], output_time_frame=cfg["Tout"],
                    st_gcnn_dropout=dropout, joints_to_consider=cfg["V"], num_feature=64, num_layers=5,
                    layout=cfg["layout"])
        m = F.DSTDGCN(**opts)
        for b in m.modules():
            if isinstance(b, F.DSTDGCB):
                randomise_fast(b)
        perturb_bn(m, gen)
        return m, opts

    # whole models (eval, calibrated BN)
    for tag in ("h36m", "3dpw"):
        cfg = CONFIGS[tag]
        T = cfg["Tin"] + cfg["Tout"]
        m, opts = build(cfg, 0.1)
        calibrate(m, lambda: synth_input(gen, 16, T, cfg["V"], cfg["Tin"]))
        x = synth_input(gen, 4, T, cfg["V"], cfg["Tin"])
        with torch.no_grad():
            y32 = m(x).numpy()
        y64 = run64(m, x)
        out[f"model_{tag}/x"] = x.numpy()
        put_outputs(out, f"model_{tag}/", y32, y64)
        out.update({f"model_{tag}/opt/{k}": np.array(v) for k, v in opts.items()})
        out.update({f"model_{tag}/sd/{k}": v for k, v in sd_numpy(m).items()})

    # one training step (forward + inverse pass, engine/prediction.py:258-290)
    # in fp64 and fp32: gradients and the updated BN running statistics
    cfg = CONFIGS["3dpw"]
    T = cfg["Tin"] + cfg["Tout"]
    m, opts = build(cfg, 0.0)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    seq = torch.randn(4, T, cfg["V"] * 3, generator=gen)
    inp = seq.clone()
    inp[:, cfg["Tin"]:] = inp[:, cfg["Tin"] - 1:cfg["Tin"]]
    inv = seq.flip(1).clone()
    inv[:, cfg["Tin"]:] = inv[:, cfg["Tin"] - 1:cfg["Tin"]]

    def step(dtype):
        mm = F.DSTDGCN(**opts)
        mm.load_state_dict(sd0)
        mm = mm.to(dtype).train()
        i, iv, s = (t.to(dtype) for t in (inp, inv, seq))
        B, T_, VC = i.shape
        loss = mpjpe_error_3d(mm(i.view(B, T_, VC // 3, 3)).reshape(B, T_, VC), s)
        loss_i = mpjpe_error_3d(mm(iv.view(B, T_, VC // 3, 3)).reshape(B, T_, VC), s.flip(1))
        all_loss = (loss + loss_i) / 2
        all_loss.backward()
        g = {k: p.grad.detach().clone() for k, p in mm.named_parameters() if p.grad is not None}
        return float(all_loss.detach()), g, {k: v.detach().clone() for k, v in mm.state_dict().items()}

    l64, g64, sd64 = step(torch.float64)
    l32, g32, _ = step(torch.float32)
    out.update({"train/inp": inp.numpy(), "train/inv": inv.numpy(), "train/seq": seq.numpy(),
                "train/loss64": np.array(l64), "train/loss32": np.array(l32)})
    out.update({f"train/opt/{k}": np.array(v) for k, v in opts.items()})
    out.update({f"train/sd0/{k}": v.numpy() for k, v in sd0.items()})
    for k in g64:
        out[f"train/g64/{k}"] = g64[k].float().numpy()  # fp64 values rounded to fp32
        out[f"train/g32err/{k}"] = np.array(float((g32[k].double() - g64[k]).abs().max()))
    for k, v in sd64.items():
        if "running_" in k:
            out[f"train/sd1/{k}"] = v.float().numpy()
    np.savez_compressed(os.path.join(HERE, "dstdgcn_fast.npz"), **out)


def main():
    torch.set_num_threads(8)
    gen = torch.Generator().manual_seed(20250725)
    torch.manual_seed(1234)
    if sys.argv[1:] == ["train"]:
        gen_train_grads(gen)
        return
    if sys.argv[1:] == ["plain"]:
        gen_plain_layers(gen)
        return
    if sys.argv[1:] == ["fast"]:
        gen_fast(gen)
        return
    gen_graphs()
    gen_ops(gen)
    gen_blocks(gen)
    gen_models(gen)
    gen_engine(gen)
    gen_train_grads(gen)
    gen_plain_layers(gen)
    gen_fast(gen)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
