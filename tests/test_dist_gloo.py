"""Multi-process (world size 2, gloo, CPU) coverage of the data-parallel path
(SURVEY §8(e)): contiguous sharding, weight broadcast that keeps the
A_s/R_s alias, ragged all-gather, metric all_reduce, and that a sharded eval
forward equals the full-batch forward (the property the GPU bench's weak
scaling rests on; the per-rank compute here is the fp64 oracle because there
is no GPU in this leg -- on the box each rank runs the HIP path)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, group, load_npz

import dstd_dist as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_numpy(v):
    # plain arrays through the queue: torch's shared-memory tensor hand-off
    # dies with the worker process
    if isinstance(v, torch.Tensor):
        return v.numpy()
    if isinstance(v, dict):
        return {k: _to_numpy(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_to_numpy(x) for x in v)
    return v


def _worker(rank, world, port, fn_name, q):
    import sys
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if ":" in fn_name:  # a body defined in another test module ("module:function")
            import importlib
            mod, fn = fn_name.split(":")
            body = getattr(importlib.import_module(mod), fn)
        else:
            body = globals()[fn_name]
        q.put((rank, _to_numpy(body(rank, world))))
    except Exception as e:  # surface worker failures in the parent
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def run_world(fn_name, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, v in res.items():
        if isinstance(v, Exception):
            raise v
    return {r: _to_torch(v) for r, v in res.items()}


def _to_torch(v):
    import numpy as np
    if isinstance(v, np.ndarray):
        return torch.from_numpy(v)
    if isinstance(v, dict):
        return {k: _to_torch(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_to_torch(x) for x in v)
    return v


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (5, 2), (2048, 8), (257, 8), (3, 4)])
def test_shard_bounds_partition(n, world):
    spans = [D.shard_bounds(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, _) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= (1 if n else 0)
    with pytest.raises(ValueError):
        D.shard_bounds(n, world, world)


# ---- per-rank bodies (run under gloo, world 2) -------------------------------
def _broadcast_body(rank, world):
    from model import DSTDGCB
    torch.manual_seed(100 + rank)  # ranks start with different weights
    blk = DSTDGCB(64, 64, 35, 22, "h36m")
    with torch.no_grad():
        for p in blk.parameters():
            p.copy_(torch.randn(p.shape))
    D.broadcast_module(blk, src=0)
    alias = blk.A_s.data_ptr() == blk.R_s.data_ptr()
    return {k: v.clone() for k, v in blk.state_dict().items()}, alias


def _gather_body(rank, world):
    n = 5
    lo, hi = D.shard_bounds(n, world, rank)
    y_local = torch.arange(lo, hi, dtype=torch.float32)[:, None].repeat(1, 3)
    full = D.gather_batch(y_local, n)
    sums, cnt = D.reduce_partials(torch.tensor([float(hi - lo), 2.0 * rank]), torch.tensor([hi - lo]))
    return full, sums, cnt


def _sharded_model_body(rank, world):
    from oracle import dstdgcn_oracle as O
    d = load_npz("model_h36m.npz")
    sd = {k: torch.from_numpy(v) for k, v in group(d, "sd/").items()}
    opts = {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}
    x = torch.from_numpy(d["x"])  # B=4 fixture batch
    y = D.sharded_forward(lambda xs: O.dstdgcn(xs, sd, opts["num_layers"]), x)
    return y, torch.from_numpy(d["y64"])


def test_broadcast_module_syncs_weights_and_keeps_alias():
    res = run_world("_broadcast_body")
    (sd0, a0), (sd1, a1) = res[0], res[1]
    assert a0 and a1
    assert sd0.keys() == sd1.keys()
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


def test_gather_batch_ragged_and_reduce_partials():
    res = run_world("_gather_body")
    for r in (0, 1):
        full, sums, cnt = res[r]
        assert torch.equal(full[:, 0], torch.arange(5, dtype=torch.float32))
        assert torch.equal(sums, torch.tensor([5.0, 2.0]))
        assert cnt.item() == 5 and cnt.dtype == torch.int64


def test_sharded_forward_equals_full_batch():
    res = run_world("_sharded_model_body")
    for r in (0, 1):
        y, y64 = res[r]
        # fp64 oracle on a shard vs the reference's fp64 output on the batch
        assert torch.allclose(y, y64.to(y.dtype), rtol=0, atol=1e-5 * float(y64.abs().max()))


def _allreduce_grads_body(rank, world):
    torch.manual_seed(7)  # same module on every rank
    lin = torch.nn.Linear(4, 3)
    frozen = torch.nn.Parameter(torch.ones(2), requires_grad=False)
    x = torch.full((5, 4), float(rank + 1))
    lin(x).sum().backward()
    local = [p.grad.clone() for p in lin.parameters()]
    D.allreduce_grads(list(lin.parameters()) + [frozen])
    return local, [p.grad.clone() for p in lin.parameters()], frozen.grad is None


def test_allreduce_grads_averages_one_bucket():
    """Data-parallel training exchange: every rank ends with the
    mean of the per-rank gradients; parameters without a gradient are skipped."""
    res = run_world("_allreduce_grads_body")
    mean = [(a + b) / 2 for a, b in zip(res[0][0], res[1][0])]
    for r in (0, 1):
        local, avg, frozen_none = res[r]
        assert frozen_none
        for m, a in zip(mean, avg):
            assert torch.allclose(m, a)
    assert not torch.allclose(res[0][0][0], res[1][0][0])


def _allreduce_arena_body(rank, world):
    import dstd_native as N
    torch.manual_seed(7)
    lin = torch.nn.Linear(4, 3)
    holder = torch.nn.Module()
    arena, direct = N.grad_sink(holder, list(lin.parameters()), "cpu")  # installs the arena views
    x = torch.full((5, 4), float(rank + 1))
    with torch.no_grad():  # what a native backward does: += into the views
        lin.weight.grad += torch.ones(3, 5) @ x
        lin.bias.grad += torch.ones(3) * 5
    local = [p.grad.clone() for p in lin.parameters()]
    D.allreduce_grads(list(lin.parameters()))
    same_base = all(p.grad._base is arena.buf for p in lin.parameters())
    return direct, local, [p.grad.clone() for p in lin.parameters()], same_base


def test_allreduce_grads_reduces_the_arena_in_place():
    """Gradients that are slices of one arena (dstd_native.grad_sink) are
    averaged by one all-reduce of the arena itself and stay views of it."""
    res = run_world("_allreduce_arena_body")
    mean = [(a + b) / 2 for a, b in zip(res[0][1], res[1][1])]
    for r in (0, 1):
        direct, local, avg, same_base = res[r]
        assert direct and same_base
        for m, a in zip(mean, avg):
            assert torch.allclose(m, a)


# ---- sharded test metric of the engine (engine/prediction.py:391-404) -------
def _engine_save_body(rank, world):
    """PredictionEngine.test(save_path=...) under torch.distributed: the ranks'
    (result, target) parts are gathered to rank 0 in loader order and written
    once (a rank without a batch contributes nothing)."""
    out = _engine_metric_body(rank, world, save_path=os.environ["DSTD_TEST_SAVE"], n_batches=int(
        os.environ.get("DSTD_TEST_BATCHES", "3")))
    return out[2]


def _engine_save_presharded_body(rank, world):
    """The same through a presharded loader: a DistributedSampler interleaves
    the samples over the ranks and pads the last with a duplicate."""
    out = _engine_metric_body(rank, world, save_path=os.environ["DSTD_TEST_SAVE"],
                              presharded=int(os.environ["DSTD_TEST_N"]))
    return out[2], out[1]


def _engine_metric_body(rank, world, save_path=None, n_batches=3, presharded=0):
    """PredictionEngine.test under torch.distributed: each rank evaluates its
    round-robin share of the loader's batches and the per-frame sums / counts
    are all-reduced.  No GPU in this leg: the model is the fp64 oracle and the
    per-batch metric the oracle's restatement of :366-404 (the native forward
    and the dstd_frame_mpjpe kernel are checked on the GPU,
    tests/test_gpu_train.py::test_engine_test_metric_matches_reference)."""
    from engine import PredictionEngine
    from oracle import dstdgcn_oracle as O
    d = load_npz("engine.npz")
    sd = group(d, "test/sd/")

    class OracleModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.anchor = torch.nn.Parameter(torch.zeros(1))  # gives the engine a device

        def forward(self, x):
            return O.dstdgcn(x, sd, 5).float()

    class CPUEngine(PredictionEngine):
        seen = []

        def _frame_metric(self, all_seqs, outputs, t_out0, used_pos, joint_src, frames, sums):
            self.seen.append(all_seqs.shape[0])
            pred = self._fill_pred(all_seqs, outputs, used_pos, joint_src, t_out0).double()
            targ = all_seqs.view(pred.shape).double()
            for k, f in enumerate(frames.tolist()):
                sums[k] += float((targ[:, f] - pred[:, f]).norm(dim=-1).mean(dim=1).sum())

    class _Log:
        def info(self, *a, **k):
            pass

    cfg = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
               loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)
    eng = CPUEngine(cfg, OracleModel(), _Log())
    inputs = torch.from_numpy(d["test/inputs"])
    all_seqs = torch.from_numpy(d["test/all_seqs"])
    # three batches (2, 1, 1): rank 0 takes batches 0 and 2, rank 1 batch 1
    loader = [(inputs[:2], None, None, all_seqs[:2]), (inputs[2:3], None, None, all_seqs[2:3]),
              (inputs[3:], None, None, all_seqs[3:])][:n_batches]
    if presharded:
        n = presharded
        ds = torch.utils.data.TensorDataset(inputs[:n], torch.zeros(n), torch.zeros(n), all_seqs[:n])
        sampler = torch.utils.data.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=False)
        loader = torch.utils.data.DataLoader(ds, batch_size=1, sampler=sampler)
    avg, metric = eng.test(loader, input_n=10, eval_frame=list(d["test/eval_frame"]), dim_used=d["test/dim_used"],
                           joint_to_ignore=d["test/joint_to_ignore"], joint_equal=d["test/joint_equal"],
                           save_path=save_path)
    return avg, metric, list(CPUEngine.seen)


def test_engine_test_metric_sharded_equals_reference():
    d = load_npz("engine.npz")
    res = run_world("_engine_metric_body")
    ref, ref_avg = d["test/metric"], float(d["test/avg"])
    assert res[0][2] == [2, 1] and res[1][2] == [1]  # the batches each rank evaluated
    for r in (0, 1):
        avg, metric, _ = res[r]
        assert float((torch.as_tensor(metric) - torch.from_numpy(ref)).abs().max()) <= 2e-4 * float(abs(ref).max())
        assert abs(avg - ref_avg) <= 2e-4 * ref_avg


@pytest.mark.parametrize("n_batches", [3, 1])
def test_engine_test_save_path_sharded(tmp_path, n_batches):
    """save_path with two ranks: one file, written by rank 0, holding every
    batch in loader order (n_batches = 1: rank 1 evaluates nothing)."""
    import numpy as np
    d = load_npz("engine.npz")
    prefix = str(tmp_path / "res")
    os.environ["DSTD_TEST_SAVE"], os.environ["DSTD_TEST_BATCHES"] = prefix, str(n_batches)
    try:
        seen = run_world("_engine_save_body")
    finally:
        del os.environ["DSTD_TEST_SAVE"], os.environ["DSTD_TEST_BATCHES"]
    assert seen[0] == ([2, 1] if n_batches == 3 else [2]) and seen[1] == ([1] if n_batches == 3 else [])
    f = np.load(prefix + ".npz")
    n = 4 if n_batches == 3 else 2
    all_seqs = d["test/all_seqs"][:n]
    assert f["target"].shape[0] == n and f["result"].shape == f["target"].shape
    np.testing.assert_array_equal(f["target"], all_seqs.reshape(n, all_seqs.shape[1], -1, 3)[:, 10:])


@pytest.mark.parametrize("n", [3, 4])
def test_engine_test_save_path_presharded(tmp_path, n):
    """save_path with a DistributedSampler loader (samples interleaved over
    the ranks; n = 3 pads rank 1 with a duplicate of sample 0): the file holds
    each sample once, in dataset order, and the metric counts each sample
    once too -- the padding duplicate stays out of the per-frame sums and the
    sample count, so both ranks report the single-process metric."""
    import numpy as np
    d = load_npz("engine.npz")
    prefix = str(tmp_path / "res")
    os.environ["DSTD_TEST_SAVE"], os.environ["DSTD_TEST_N"] = prefix, str(n)
    try:
        res = run_world("_engine_save_presharded_body")
    finally:
        del os.environ["DSTD_TEST_SAVE"], os.environ["DSTD_TEST_N"]
    seen = {r: v[0] for r, v in res.items()}
    # the batches each rank put into the metric (rank 1's padding batch: none)
    assert seen[0] == [1, 1] and seen[1] == ([1] if n == 3 else [1, 1])
    _, single, _ = _engine_metric_body(0, 1, presharded=n)  # one process, same sampler
    for r in (0, 1):
        np.testing.assert_allclose(np.asarray(res[r][1]), np.asarray(single), rtol=1e-6)  # fp32 sums, other order
    f = np.load(prefix + ".npz")
    all_seqs = d["test/all_seqs"][:n]
    np.testing.assert_array_equal(f["target"], all_seqs.reshape(n, all_seqs.shape[1], -1, 3)[:, 10:])
    assert f["result"].shape == f["target"].shape
