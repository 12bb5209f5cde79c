"""Data-parallel sharding of the eval forward.

One process per GPU (``torch.distributed`` over RCCL; ``gloo`` in the CPU
tests).  The DSTDGCN eval forward has no cross-sample coupling -- BatchNorm uses
running statistics (``model/dstdgcn.py:35-50``), dropout is off, no op reduces
over the batch -- so a global batch is partitioned into contiguous per-rank
shards and each rank runs its shard alone: there is no exchange inside the
forward.  The only collectives are outside it:

* ``broadcast_module``  -- weights once, rank ``src`` -> all (~0.9 MB);
* ``gather_batch``      -- per-rank outputs back to one tensor when a caller
                           needs the whole batch (parity checks, export);
* ``reduce_partials``   -- metric partial sums / counts (``all_reduce(SUM)``),
                           e.g. the per-frame MPJPE sums of the test metric
                           (``engine/prediction.py:366-404``).

Training (config 5) has one real exchange per step: the data-parallel
gradient average, ``allreduce_grads`` -- one flat bucket (~0.75 MB for the
3DPW model), a single ring all-reduce over xGMI.  Train-mode BatchNorm keeps
per-rank batch statistics (the DDP default) unless ``convert_sync_batchnorm``
opts the model into cross-rank BatchNorm (SURVEY §8(e) SyncBN: every BatchNorm
of the native train forward normalises with all ranks' statistics -- one
all-gather of (mean, M2, count) per BatchNorm forward, one all-reduce of
(sum dz, sum dz*xhat) per BatchNorm backward, issued by the library through
``BnSync``'s collective on the call's stream).
"""
import ctypes
import sys

import torch
import torch.distributed as dist

import dstd_native as native


def shard_bounds(n, world, rank):
    """Contiguous shard ``[lo, hi)`` of ``n`` samples for ``rank``: the first
    ``n % world`` ranks hold one extra sample, so shards differ by at most one
    and concatenating them in rank order restores the batch."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard(x, world, rank, dim=0):
    lo, hi = shard_bounds(x.shape[dim], world, rank)
    return x.narrow(dim, lo, hi - lo)


def broadcast_module(module, src=0, group=None):
    """Broadcast every parameter and buffer of ``module`` from ``src`` in place.
    Tensors sharing storage (the reference's ``A_s``/``R_s`` alias,
    ``model/dstdgcn.py:107-109``) are sent once, so the alias survives.  The
    collectives write the tensors outside autograd's version counters, so the
    native modules' cached folded constants are invalidated explicitly."""
    from model.dstdgcn import invalidate_native_cache
    seen = set()
    for t in list(module.parameters()) + list(module.buffers()):
        key = (t.untyped_storage().data_ptr(), t.storage_offset(), tuple(t.shape))
        if key in seen:
            continue
        seen.add(key)
        with torch.no_grad():
            dist.broadcast(t, src=src, group=group)
    invalidate_native_cache(module)


def gather_batch(y_local, n_total, group=None):
    """All-gather per-rank shards (``shard_bounds`` layout, dim 0) into the full
    ``[n_total, ...]`` batch on every rank.  Ragged shards are padded to the
    largest shard for the collective and trimmed afterwards."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(n_total, world, rank)
    if y_local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: shard has {y_local.shape[0]} samples, expected {hi - lo}")
    cap = shard_bounds(n_total, world, 0)[1]
    pad = y_local.new_zeros((cap,) + tuple(y_local.shape[1:]))
    pad[:hi - lo] = y_local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad.contiguous(), group=group)
    parts = []
    for r in range(world):
        a, b = shard_bounds(n_total, world, r)
        parts.append(bufs[r][:b - a])
    return torch.cat(parts, 0)


def reduce_partials(*tensors, group=None):
    """``all_reduce(SUM)`` of metric partials in one collective (the tensors
    are packed into one fp64 buffer); returns the reduced tensors."""
    flat = torch.cat([t.reshape(-1).to(torch.float64) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    out, off = [], 0
    for t in tensors:
        out.append(flat[off:off + t.numel()].reshape(t.shape).to(t.dtype))
        off += t.numel()
    return out


def sharded_forward(fn, x_full, group=None, gather=True):
    """Run ``fn`` on this rank's shard of ``x_full``; optionally gather."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    y = fn(shard(x_full, world, rank))
    return gather_batch(y, x_full.shape[0], group=group) if gather else y


def allreduce_grads(params, group=None):
    """Average ``.grad`` of ``params`` over the ranks with ONE all-reduce of a
    flat fp32 bucket (the whole model's gradient is under 1 MB, far below any
    useful bucket split on xGMI).  Parameters without a gradient are skipped
    (identically on every rank: the set only depends on requires_grad)."""
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if p.grad is not None]
    if world == 1 or not grads:
        return
    base = grads[0]._base
    if base is not None and base.dim() == 1 and all(g._base is base for g in grads):
        # the gradients are slices of one arena (dstd_native.grad_sink): reduce
        # it in place, padding gaps included (zeros on every rank)
        dist.all_reduce(base, op=dist.ReduceOp.SUM, group=group)
        base.div_(world)
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world)
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()


class BnSync:
    """The dstd_bn_sync of one model (include/dstd_gcn_train.h): this rank's
    place in ``group``, a device buffer sized by dstd_bn_sync_buffer_floats,
    and the collective the library calls at every BatchNorm -- an all-gather
    of the per-rank statistics (forward) or an all-reduce of the gradient
    sums (backward) over torch.distributed on the current stream (RCCL / NCCL
    in place on the device; gloo through host copies)."""

    def __init__(self, num_feature, V, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        n = native.lib().dstd_bn_sync_buffer_floats(self.world, num_feature, V)
        self.buf = torch.zeros(n, dtype=torch.float32, device=device)
        self.host = dist.get_backend(group) == "gloo" and self.buf.is_cuda
        self._fn = native.COLLECTIVE_FN(self._collective)  # kept alive with the struct
        self._s = native.BnSyncStruct(self.world, self.rank, self._fn, None, self.buf.data_ptr(), n)
        self.calls = 0
        self._ext = {}  # ExternalStream per foreign stream handle

    def struct_ref(self):
        return ctypes.byref(self._s)

    def _stream_ctx(self, stream):
        """torch's stream context for the library's call stream (the header's
        contract: the collective is ordered on ``stream``), a no-op when it
        already is torch's current stream (every native call site today)."""
        import contextlib
        if not self.buf.is_cuda:
            return contextlib.nullcontext()
        dev = self.buf.device
        handle = stream or 0
        if handle == torch.cuda.current_stream(dev).cuda_stream:
            return contextlib.nullcontext()
        if handle == 0:
            return torch.cuda.stream(torch.cuda.default_stream(dev))
        ext = self._ext.get(handle)
        if ext is None:
            ext = self._ext[handle] = torch.cuda.ExternalStream(handle, device=dev)
        return torch.cuda.stream(ext)

    def _collective(self, ctx, op, buf, count, stream):
        try:
            with self._stream_ctx(stream):
                return self._collective_on_stream(op, buf, count)
        except Exception as e:  # the library returns DSTD_ECOLLECTIVE
            print(f"dstd_bn_sync collective failed: {e!r}", file=sys.stderr)
            return 1

    def _collective_on_stream(self, op, buf, count):
        if buf != self.buf.data_ptr():
            raise RuntimeError("dstd_bn_sync: foreign buffer")
        self.calls += 1
        if op == native.COLL_ALLGATHER:
            out = self.buf[:count * self.world]
            mine = out[self.rank * count:(self.rank + 1) * count].clone()
            if self.host:
                o = torch.empty(out.shape, dtype=out.dtype)
                dist.all_gather_into_tensor(o, mine.cpu(), group=self.group)
                out.copy_(o)
            else:
                dist.all_gather_into_tensor(out, mine, group=self.group)
        elif op == native.COLL_ALLREDUCE_SUM:
            t = self.buf[:count]
            if self.host:
                c = t.cpu()
                dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
                t.copy_(c)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        else:
            raise ValueError(f"dstd_bn_sync: unknown collective {op}")
        return 0


def convert_sync_batchnorm(model, group=None):
    """Opt ``model`` (a DSTDGCN on its device, in a process group) into
    cross-rank BatchNorm for its native train-mode forward and backward --
    torch.nn.SyncBatchNorm.convert_sync_batchnorm's semantics without
    replacing modules (the state-dict schema is unchanged).  Returns the
    model; ``model._dstd_bn_sync = None`` goes back to per-rank statistics."""
    dev = next(model.parameters()).device
    model._dstd_bn_sync = BnSync(model.num_feature, model.joints_to_consider, dev, group)
    return model
