"""The data-parallel path with the NATIVE model in more than one
process: two ranks share the box's one GPU and talk over gloo on GPU tensors
(RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's).

* config 4 (sharded eval): dstd_dist.sharded_forward of the native forward,
  all-gathered, is bit-identical to the full-batch forward on every rank
  (eval BatchNorm uses running statistics: no cross-sample coupling), after
  the weights went out from rank 0 with broadcast_module;
* config 5 (data-parallel training): one PredictionEngine.train step on each
  rank's half of the batch, whose allreduce_grads reduces the native gradient
  arena in place, hands Adam exactly the mean of the two ranks' own
  single-process gradients (engine/prediction.py:198-317, 391-404)."""
import pytest
import torch

from conftest import group, load_npz
from test_dist_gloo import run_world

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _h36m_model():
    from model import get_model
    d = load_npz("model_h36m.npz")
    opts = {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "sd/").items()})
    return m.to(DEV).eval(), opts


def _sharded_native_body(rank, world):
    import dstd_dist as D
    torch.cuda.set_device(0)
    m, opts = _h36m_model()
    if rank != 0:  # rank 1 starts from other weights; the broadcast must fix them
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(0.5)
    D.broadcast_module(m, src=0)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    g = torch.Generator().manual_seed(21)
    x = torch.randn(11, T, 22, 3, generator=g)  # ragged shards: 6 + 5
    x[:, opts["input_time_frame"]:] = x[:, opts["input_time_frame"] - 1:opts["input_time_frame"]]
    x = x.to(DEV)
    with torch.no_grad():
        y_sh = D.sharded_forward(m, x)
        y_full = m(x)
    torch.cuda.synchronize()
    return {"equal": bool(torch.equal(y_sh, y_full)), "y": y_sh.cpu(),
            "alias": m.conv_st_in.stgcn[0][0].A_s.data_ptr() == m.conv_st_in.stgcn[0][0].R_s.data_ptr()}


def test_sharded_native_forward_equals_full_batch():
    res = run_world("test_gpu_dist:_sharded_native_body")
    for r in (0, 1):
        assert res[r]["equal"], r
    assert torch.equal(res[0]["y"], res[1]["y"])


def _model_3dpw():
    from model import get_model
    from model.dstdgcn import DSTDGCB
    d = load_npz("engine.npz")
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "train/sd0/").items()})
    m = m.to(DEV)
    for b in m.modules():  # the CPU fixture's A_s/R_s alias (test_gpu_train._realias)
        if isinstance(b, DSTDGCB):
            b.A_s.data = b.R_s.data
    return m.train(), d


def _dp_train_body(rank, world):
    import torch.distributed as dist

    import dstd_dist as D
    from engine import PredictionEngine
    torch.cuda.set_device(0)

    class _Log:
        def info(self, *a, **k):
            pass

    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    d = load_npz("engine.npz")
    batch = tuple(D.shard(torch.from_numpy(d[f"train/{n}0"]), world, rank).contiguous()
                  for n in ("inp", "inv", "seq", "seq"))

    # (1) this rank's own single-process gradient of its shard: the engine's
    # step with the all-reduce left out (the process group is up, so take the
    # single-process branch by hand)
    m1, _ = _model_3dpw()
    eng1 = PredictionEngine(cfg, m1, _Log())
    local = {}
    eng1.optimizer.step = lambda: local.update(
        {n: p.grad.detach().clone() for n, p in m1.named_parameters() if p.grad is not None})
    import engine.prediction as EP
    saved_world = EP._world
    EP._world = lambda: (0, 1)
    try:
        eng1.train([batch], 0, max_iter=1)
    finally:
        EP._world = saved_world

    # (2) the data-parallel step: allreduce_grads over the native arena
    m2, _ = _model_3dpw()
    eng2 = PredictionEngine(cfg, m2, _Log())
    seen = {}
    step = eng2.optimizer.step

    def capture():
        seen.update({n: p.grad.detach().clone() for n, p in m2.named_parameters() if p.grad is not None})
        seen["_arena"] = getattr(m2, "_dstd_grad_arena", None) is not None and all(
            p.grad._base is m2._dstd_grad_arena.buf for p in m2.parameters() if p.grad is not None)
        return step()

    eng2.optimizer.step = capture
    eng2.train([batch], 0, max_iter=1)
    # the mean of the two ranks' own gradients, over the same gloo group
    names = sorted(local)
    flat = torch.cat([local[n].reshape(-1) for n in names])
    both = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(both, flat)
    mean = (both[0] + both[1]) / 2
    got = torch.cat([seen[n].reshape(-1) for n in names])
    return {"equal": bool(torch.equal(got, mean)), "maxdiff": float((got - mean).abs().max()),
            "arena": bool(seen["_arena"]), "n": len(names),
            "differs": bool(not torch.equal(both[0], both[1]))}


def test_dp_training_step_averages_native_arena():
    res = run_world("test_gpu_dist:_dp_train_body")
    for r in (0, 1):
        assert res[r]["arena"], "the engine's gradients were not slices of the native arena"
        assert res[r]["differs"], "the two shards gave the same gradient: the test would prove nothing"
        assert res[r]["equal"], (r, res[r]["maxdiff"])


def _syncbn_step(rank, world, sync):
    """One engine step (forward pair, two losses, native backward, the
    data-parallel gradient average) on this rank's half of the fixture batch,
    with cross-rank BatchNorm (dstd_dist.convert_sync_batchnorm) or per-rank;
    returns the averaged gradients and the buffers after the step."""
    import dstd_dist as D
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    d = load_npz("engine.npz")
    batch = tuple(D.shard(torch.from_numpy(d[f"train/{n}0"]), world, rank).contiguous()
                  for n in ("inp", "inv", "seq", "seq"))
    m, _ = _model_3dpw()
    if sync:
        D.convert_sync_batchnorm(m)
    eng = PredictionEngine(cfg, m, _Log())
    seen = {}
    step = eng.optimizer.step

    def capture():
        seen.update({n: p.grad.detach().clone().cpu() for n, p in m.named_parameters() if p.grad is not None})
        return step()

    eng.optimizer.step = capture
    eng.train([batch], 0, max_iter=1)
    bufs = {n: b.detach().clone().cpu() for n, b in m.named_buffers()}
    return seen, bufs, (m._dstd_bn_sync.calls if sync else 0)


def _syncbn_body(rank, world):
    torch.cuda.set_device(0)
    g_sync, b_sync, calls = _syncbn_step(rank, world, True)
    g_local, _, _ = _syncbn_step(rank, world, False)
    return {"g_sync": g_sync, "b_sync": b_sync, "g_local": g_local, "calls": calls}


def test_syncbn_dp_step_equals_full_batch_step():
    """SURVEY §8(e) SyncBN: the two-rank data-parallel step with cross-rank
    BatchNorm is the step of ONE process on the whole batch, while per-rank
    BatchNorm is not.  Gradients: against the CPU oracle's fp64 step on the
    full batch (tests/test_oracle_golden.py pins it to the reference's own
    fp64 gradients), with the whole-model criterion of tests/test_gpu_train.py
    (check_ratios: every tensor within 3x -- the global sums 4x -- of its measured fp32 noise floor --
    fp32_noise: the fp32 oracle over several implementations and sample
    orders, and the reference's own fp32 run), for the single-process native
    step and for both ranks.  Running statistics within 1e-4 of the
    single-process native step's."""
    import engine.prediction as EP
    from oracle import dstdgcn_oracle as O
    from test_gpu_train import check_ratios, fp32_noise, noise_ratios
    res = run_world("test_gpu_dist:_syncbn_body")
    # the single-process native step on the full batch of 8
    from engine import PredictionEngine

    class _Log:
        def info(self, *a, **k):
            pass

    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    d = load_npz("engine.npz")
    batch = tuple(torch.from_numpy(d[f"train/{n}0"]) for n in ("inp", "inv", "seq", "seq"))
    m, _ = _model_3dpw()
    eng = PredictionEngine(cfg, m, _Log())
    ref = {}
    step = eng.optimizer.step
    eng.optimizer.step = lambda: (ref.update({n: p.grad.detach().clone().cpu() for n, p in m.named_parameters()
                                              if p.grad is not None}), step())[1]
    saved_world = EP._world
    EP._world = lambda: (0, 1)
    try:
        eng.train([batch], 0, max_iter=1)
    finally:
        EP._world = saved_world
    ref_bufs = {n: b.detach().clone().cpu() for n, b in m.named_buffers()}
    # the oracle's fp64 step on the full batch and the fp32 noise floor
    sd0 = group(d, "train/sd0/")
    batch_np = tuple(d[f"train/{n}0"] for n in ("inp", "inv", "seq"))
    P = O.train_params(sd0, torch.float64, DEV)
    _, lall = O.step_loss(P, batch_np, 5)
    lall.backward()
    g64 = {k: v.grad.double().cpu().numpy() for k, v in P.items() if v.grad is not None}
    assert set(g64) == set(ref), "the engine step and the oracle step differ in their trainable set"
    gr = load_npz("train_grads.npz")
    noise = fp32_noise(sd0, batch_np, g64, extra={k: gr["g32err/" + k] for k in g64})
    check_ratios(noise_ratios(ref, g64, noise), "single process")
    for r in (0, 1):
        # 15 BatchNorms x (forward all-gather, backward all-reduce) per model call
        assert res[r]["calls"] > 0
        check_ratios(noise_ratios(res[r]["g_sync"], g64, noise), f"rank {r} SyncBN")
        for n, b in ref_bufs.items():
            if n.endswith("num_batches_tracked"):
                assert int(res[r]["b_sync"][n]) == int(b), n
            else:
                # (1e-4: the statistics are fp32 Chan merges of the ranks' partials
                # against the full batch's own partition -- measured up to 1.3e-5
                # of the largest running variance, ~1.2e3 after the encoders)
                assert float((res[r]["b_sync"][n] - b).abs().max()) <= 1e-4 * max(float(b.abs().max()), 1e-6), n
    import numpy as np
    loc = np.median([v for v, _ in noise_ratios(res[0]["g_local"], g64, noise)])
    print("per-rank BatchNorm: median err / noise floor", loc)
    assert loc > 10.0, ("per-rank BatchNorm met the full-batch bar: the test would prove nothing", loc)

class _FailingSync:
    """A one-rank dstd_bn_sync whose collective fails at the n-th backward
    all-reduce (the forward all-gathers succeed: with one rank they move
    nothing) -- DSTD_ECOLLECTIVE in the middle of the model backward, after
    the weight-gradient stream has been forked."""

    def __init__(self, model, fail_at):
        import dstd_native as native
        n = native.lib().dstd_bn_sync_buffer_floats(1, model.num_feature, model.joints_to_consider)
        self.buf = torch.zeros(n, dtype=torch.float32, device=DEV)
        self.fail_at, self.reduces = fail_at, 0
        self._fn = native.COLLECTIVE_FN(self._collective)
        self._s = native.BnSyncStruct(1, 0, self._fn, None, self.buf.data_ptr(), n)
        self.calls = 0

    def struct_ref(self):
        import ctypes
        return ctypes.byref(self._s)

    def _collective(self, ctx, op, buf, count, stream):
        import dstd_native as native
        self.calls += 1
        if op == native.COLL_ALLREDUCE_SUM:
            self.reduces += 1
            if self.reduces == self.fail_at:
                return 1
        return 0


def test_backward_error_after_fork_joins_the_side_stream():
    """an error return from the model backward after the weight-
    gradient stream was forked (a SyncBN collective failing mid-backward)
    must still order the side stream's work before the caller's stream
    (Wgrad's destructor joins it).  The failing call raises naming the entry
    point; afterwards the device is healthy and a plain step on a fresh model
    reproduces the reference step bit for bit."""
    from engine import mpjpe_error_3d

    def step(m):
        g = torch.Generator().manual_seed(5)
        seq = (0.6 * torch.randn(32, 40, 69, generator=g)).to(DEV)
        inp = seq.clone()
        inp[:, 10:] = inp[:, 9:10]
        y = m(inp.view(32, 40, 23, 3)).view(32, 40, 69)
        mpjpe_error_3d(y, seq).backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}

    m0, _ = _model_3dpw()
    want = step(m0)
    for fail_at in (3, 15):  # an early and a late BatchNorm of the backward
        m, _ = _model_3dpw()
        m._dstd_bn_sync = _FailingSync(m, fail_at)
        with pytest.raises(RuntimeError, match="dstd_model_train_bwd_sync"):
            step(m)
        assert m._dstd_bn_sync.reduces == fail_at
        torch.cuda.synchronize()
    m1, _ = _model_3dpw()
    got = step(m1)
    for n in want:
        assert torch.equal(got[n], want[n]), n
