"""BASELINE configs 4 and 5 at their own shapes, eight ranks on
the box's one GPU: eight processes over gloo, each running the NATIVE path on
cuda:0 (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the
driver's).  What differs from the 8xMI355X run is only the transport of the
collectives, not what is sharded, reduced or computed.

* config 4 -- H36M B=2048 sharded 256 per rank x 8 (dstd_dist.sharded_forward):
  the gathered output is bit-identical to the single-process B=2048 forward,
  the engine's per-frame test metric over eight 256-sequence batches (one per
  rank, all-reduced) equals the single-process metric, and sampled sequences
  meet the whole-model bar against the fp64 oracle;
* config 5 -- 3DPW training at 32 per rank (global 256,
  configs/dstdgcn/dstdgcn_3dpw.yaml:19) with cross-rank BatchNorm: one
  PredictionEngine.train step (engine/prediction.py:198-317) gives every rank
  the same gradients, which meet the single-process B=256 step's criterion
  against the oracle's fp64 step (tests/test_gpu_train.py
  test_model_step_gradients_at_training_batch), and running statistics within
  1e-4 of the single-process step's."""
import numpy as np
import pytest
import torch

from conftest import group, load_npz, model_tol, rel_err
from test_dist_gloo import run_world

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
WORLD = 8
EVAL_FRAME = [1, 3, 7, 9, 13, 24]  # H36M 80/160/320/400/560/1000 ms at 25 fps


class _Log:
    def info(self, *a, **k):
        pass


def _cfg():
    return dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
                loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)


# ---- config 4 ---------------------------------------------------------------
def _config4_inputs(opts):
    import bench
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(2048, T, 22, opts["input_time_frame"], 2048)
    g = torch.Generator().manual_seed(4)
    all_seqs = x.reshape(2048, T, 66) + 0.05 * torch.randn(2048, T, 66, generator=g)
    return x, all_seqs


def _config4_body(rank, world):
    import torch.distributed as dist

    import dstd_dist as D
    import engine.prediction as EP
    from engine import PredictionEngine
    from test_gpu_dist import _h36m_model
    torch.cuda.set_device(0)
    m, opts = _h36m_model()
    if rank != 0:  # the broadcast must replace these
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(0.5)
    D.broadcast_module(m, src=0)
    x, all_seqs = _config4_inputs(opts)
    xd = x.to(DEV)
    with torch.no_grad():
        y_sh = D.sharded_forward(m, xd)  # this rank's 256, all-gathered
        y_full = m(xd) if rank == 0 else torch.empty_like(xd)
    dist.broadcast(y_full, src=0)
    torch.cuda.synchronize()
    out = {"equal": bool(torch.equal(y_sh, y_full)), "shard": D.shard_bounds(2048, world, rank)}
    # the engine's test metric: 8 batches of 256, round-robin (batch r on rank r)
    loader = [(x[i * 256:(i + 1) * 256].reshape(256, -1, 66), None, None, all_seqs[i * 256:(i + 1) * 256])
              for i in range(8)]
    eng = PredictionEngine(_cfg(), m, _Log())
    out["metric"] = eng.test(loader, input_n=opts["input_time_frame"], eval_frame=EVAL_FRAME)[1]
    if rank == 0:  # the single-process metric over the same loader
        saved = EP._world
        EP._world = lambda: (0, 1)
        try:
            out["metric1"] = eng.test(loader, input_n=opts["input_time_frame"], eval_frame=EVAL_FRAME)[1]
        finally:
            EP._world = saved
        picks = [0, 255, 256, 1023, 1800, 2047]  # first / last of shards and inside them
        out["picks"] = picks
        out["y_picks"] = y_full[picks].cpu()
    return out


def test_config4_h36m_b2048_sharded_over_8_ranks():
    from oracle import dstdgcn_oracle as O
    res = run_world("test_gpu_dp8:_config4_body", world=WORLD)
    spans = [tuple(res[r]["shard"]) for r in range(WORLD)]
    assert spans == [(256 * r, 256 * (r + 1)) for r in range(WORLD)]  # 256 per rank
    for r in range(WORLD):
        assert res[r]["equal"], f"rank {r}: gathered shards differ from the B=2048 forward"
    # the all-reduced per-frame metric: every rank reports the whole loader's
    m1 = np.asarray(res[0]["metric1"])
    for r in range(WORLD):
        np.testing.assert_allclose(np.asarray(res[r]["metric"]), m1, rtol=1e-6)  # fp32 sums, other order
    # sampled sequences against the fp64 oracle at the whole-model bar
    d = load_npz("model_h36m.npz")
    sd = group(d, "sd/")
    opts = {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}
    x, _ = _config4_inputs(opts)
    picks = list(res[0]["picks"])
    y64 = O.dstdgcn(x[picks], sd, opts["num_layers"]).numpy()
    ref32 = rel_err(O.dstdgcn(x[picks], sd, opts["num_layers"], dtype=torch.float32).numpy(), y64)
    err = rel_err(np.asarray(res[0]["y_picks"]), y64)
    print(f"config 4 picks: err {err:.3e}, ref32 {ref32:.3e}")
    assert err <= model_tol(max(ref32, float(d["ref32_err"]))), (err, ref32)


# ---- config 5 ---------------------------------------------------------------
def _config5_batch():
    g = torch.Generator().manual_seed(1000 + 256)
    T, VC = 40, 69
    seq = 0.6 * torch.randn(256, T, VC, generator=g)  # the fixture batches' scale
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]  # future frames = the last observed one
    inv = seq.flip(1).clone()
    inv[:, 10:] = inv[:, 9:10]
    return inp, inv, seq


def _engine_step(m, batch, single_process=False):
    import engine.prediction as EP
    from engine import PredictionEngine
    eng = PredictionEngine(_cfg(), m, _Log())
    seen = {}
    step = eng.optimizer.step

    def capture():
        seen.update({n: p.grad.detach().clone().cpu() for n, p in m.named_parameters() if p.grad is not None})
        return step()

    eng.optimizer.step = capture
    saved = EP._world
    if single_process:
        EP._world = lambda: (0, 1)
    try:
        eng.train([batch], 0, max_iter=1)
    finally:
        EP._world = saved
    return seen, {n: b.detach().clone().cpu() for n, b in m.named_buffers()}


def _config5_body(rank, world):
    import dstd_dist as D
    from test_gpu_dist import _model_3dpw
    torch.cuda.set_device(0)
    inp, inv, seq = _config5_batch()
    batch = tuple(D.shard(t, world, rank).contiguous() for t in (inp, inv, seq, seq))
    assert batch[0].shape[0] == 32
    m, _ = _model_3dpw()
    D.convert_sync_batchnorm(m)
    grads, bufs = _engine_step(m, batch)
    return {"grads": grads, "bufs": bufs, "calls": m._dstd_bn_sync.calls}


def test_config5_3dpw_training_32_per_rank_x8_syncbn():
    from oracle import dstdgcn_oracle as O
    from test_gpu_dist import _model_3dpw
    from test_gpu_train import check_ratios, fp32_noise, noise_ratios
    res = run_world("test_gpu_dp8:_config5_body", world=WORLD)
    inp, inv, seq = _config5_batch()
    # control: the single-process native step on the whole B=256 batch
    m, d = _model_3dpw()
    ref, ref_bufs = _engine_step(m, (inp, inv, seq, seq), single_process=True)
    # the oracle's fp64 step on the whole batch and the fp32 noise floor
    sd0 = group(d, "train/sd0/")
    batch_np = (inp.numpy(), inv.numpy(), seq.numpy())
    P = O.train_params(sd0, torch.float64, DEV)
    _, lall = O.step_loss(P, batch_np, 5)
    lall.backward()
    g64 = {k: v.grad.double().cpu().numpy() for k, v in P.items() if v.grad is not None}
    assert set(g64) == set(ref)
    noise = fp32_noise(sd0, batch_np, g64)
    # the single-process step's own criterion (test_model_step_gradients_at_training_batch)
    check_ratios(noise_ratios(ref, g64, noise), "single process B=256")
    for r in range(WORLD):
        # 15 BatchNorms, forward all-gather + backward all-reduce, one forward pair
        assert res[r]["calls"] >= 30, res[r]["calls"]
        for k in ref:  # the all-reduced arena: every rank holds the same gradients
            assert torch.equal(res[r]["grads"][k], res[0]["grads"][k]), (r, k)
    check_ratios(noise_ratios(res[0]["grads"], g64, noise), "8 ranks x 32, SyncBN")
    for r in range(WORLD):
        for n, b in ref_bufs.items():
            got = res[r]["bufs"][n]
            if n.endswith("num_batches_tracked"):
                assert int(got) == int(b), n
            else:
                assert float((got - b).abs().max()) <= 1e-4 * max(float(b.abs().max()), 1e-6), (r, n)
