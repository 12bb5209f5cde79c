"""DSTD-GCN modules backed by the MI355X kernels.

Drop-in replacements for the reference's ``model/dstdgcn.py``: the same class
names, constructor signatures, sub-module names, parameter names / shapes /
registration order (so ``state_dict`` keys and optimizer state line up with
checkpoints of the reference), the same initialisation and the same A_s/R_s
storage alias (reference :107-109).  Forward passes run through the C ABI in
include/dstd_gcn.h:

  DSTDGC.forward   -> dstd_dstdgc_fwd   (reference :80-94)
  DSTDGCB.forward  -> dstd_block_fwd    (reference :141-163)
  DSTDGCN.forward  -> dstd_model_fwd    (reference :293-317)

Training runs through include/dstd_gcn_train.h:

  DSTDGC  with autograd       -> dstd_dstdgc_train_fwd / _bwd
  DSTDGCB in train mode       -> dstd_block_train_fwd / _bwd (batch-stat BN)
  DSTDGCN in train mode       -> dstd_model_train_fwd / _bwd

each wrapped in a torch.autograd.Function whose backward is the native
backward, with the reference's gradient semantics (A_s / A_t constant, R_s
aliasing A_s's storage, alpha_sm shared by both spatial convs).

There is no CPU / eager fallback: a tensor off the GPU or a missing library
raises.  An eval-mode DSTDGCB / DSTDGCN forward that autograd will
differentiate (grad enabled and an input or parameter requiring grad) runs
the native training path with BatchNorm on its running statistics
(include/dstd_gcn_train.h DSTD_TRAIN_RUNNING_STATS), as the reference
back-propagates through its eval-mode modules; under torch.no_grad() (or
with frozen parameters and input) eval runs the fused inference kernels.
"""
import itertools
import operator
import math
import weakref
from typing import List, Tuple

import numpy as np
import torch
import torch.nn as nn

import dstd_native as native

from .layers.graph import Graph
from .layers.time import Time


def conv_init(conv):
    """kaiming-normal fan_out weights, zero bias (reference :14-18)."""
    if conv.weight is not None:
        nn.init.kaiming_normal_(conv.weight, mode="fan_out")
    if conv.bias is not None:
        nn.init.constant_(conv.bias, 0)


def bn_init(bn, scale):
    nn.init.constant_(bn.weight, scale)
    nn.init.constant_(bn.bias, 0)


def weights_init(m):
    """Applied by ST_GCNN_layer to every Conv* module (reference :26-32)."""
    if "Conv" in type(m).__name__ and isinstance(getattr(m, "weight", None), torch.Tensor):
        nn.init.kaiming_normal_(m.weight, mode="fan_out")
        if isinstance(getattr(m, "bias", None), torch.Tensor):
            nn.init.constant_(m.bias, 0)


class _ForwardOnly(torch.autograd.Function):
    """Empty-batch outputs: forward is identity, backward gives the zero
    gradients torch's own ops would (nothing flows through an empty batch)."""

    @staticmethod
    def forward(ctx, y, *deps):
        ctx.shapes = [(d.shape, d.dtype, d.device) for d in deps]
        return y

    @staticmethod
    def backward(ctx, dy, *rest):
        return (dy, *[torch.zeros(sh, dtype=dt, device=dev) for sh, dt, dev in ctx.shapes])


# Native modules carry an instance token that is never reused (unlike id()):
# part of the constant-reuse tag of DSTDGCN, and the key under which the
# torch.library ops below find the module that lays out their C parameter
# struct.  Copies (deepcopy / unpickling) get a token of their own.
_UIDS = itertools.count(1)
_INSTANCES = weakref.WeakValueDictionary()


def _register(mod):
    mod._dstd_uid = next(_UIDS)
    _INSTANCES[mod._dstd_uid] = mod


class _NativeModule(nn.Module):
    # extra per-call launch-schedule flags of the eval forwards (include/dstd_gcn.h
    # DSTD_FWD_SEPARATE_ADJ / DSTD_FWD_FUSED_TEMPORAL: same results, for tests and A/B)
    _dstd_fwd_flags = 0

    def __setstate__(self, state):
        super().__setstate__(state)
        _register(self)

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        _bump_epoch()  # may have put new Parameter objects into _parameters
        return out


def invalidate_native_cache(module):
    """Force the next eval forward of every native module in ``module``'s tree
    to refold its constants.  Needed after writes the version counters do not
    see: through ``.data``, by collectives (dstd_dist.broadcast_module calls
    it), or by foreign kernels.  In-place torch ops, optimizer steps,
    ``load_state_dict`` and ``.to()`` are detected without it."""
    for m in module.modules():
        if hasattr(m, "_dstd_gen"):
            m._dstd_gen += 1


def _mark(y, *deps):
    if torch.is_grad_enabled():
        req = [d for d in deps if isinstance(d, torch.Tensor) and d.requires_grad]
        if req:
            return _ForwardOnly.apply(y, *req)
    return y


# Structure epoch: bumped by torch's global registration hooks whenever ANY
# module registers (or replaces) a parameter, buffer or submodule -- the
# assignments nn.Module.__setattr__ / register_* make -- and by
# _NativeModule._apply (.to(), .cuda(), .float() may put new Parameter objects
# straight into _parameters).  A cached walk of a native module tree is valid
# while the epoch it was taken at is current: an O(1) check per call instead
# of one identity check per (module, name, tensor) entry.
_STRUCT_EPOCH = [0]


def _bump_epoch(*args, **kwargs):
    _STRUCT_EPOCH[0] += 1


for _reg in ("register_module_parameter_registration_hook", "register_module_buffer_registration_hook",
             "register_module_module_registration_hook"):
    getattr(torch.nn.modules.module, _reg)(_bump_epoch)


def _hook_swap_tensor():
    """torch.func.functional_call and torch.nn.utils.stateless swap tensors
    into ``module._parameters`` / ``_buffers`` directly (the accessor's
    swap_tensor), past the registration hooks: bump the epoch there too, so a
    cached walk never hands the native kernels the module's own tensors in
    place of the swapped-in ones."""
    import torch.nn.utils._named_member_accessor as acc
    orig = acc.swap_tensor
    if getattr(orig, "_dstd_epoch", False):
        return

    def swap_tensor(*args, **kwargs):
        _STRUCT_EPOCH[0] += 1
        return orig(*args, **kwargs)

    swap_tensor._dstd_epoch = True
    acc.swap_tensor = swap_tensor


_hook_swap_tensor()


class _TensorTree:
    """``list(root.parameters())`` and ``list(root.buffers())`` without
    torch's generator walk of the module tree (~1.3 ms for DSTDGCN's ~350
    modules, paid per forward and per backward).  The walk is reused while the
    structure epoch it was taken at is current (no module anywhere registered
    or replaced a parameter, buffer or submodule since); a stale epoch falls
    back to checking every (parent, name, child) edge and (module, name,
    tensor) entry the walk saw, and walks again only if one of them changed."""

    def __init__(self):
        self.edges = self.pents = self.bents = None
        self.params = self.buffers = None
        self.epoch = -1

    def _walk(self, root):
        mods, edges, seen = [], [], set()

        def rec(mod):
            seen.add(id(mod))
            mods.append(mod)
            for name, child in mod._modules.items():
                edges.append((mod, name, child))
                if child is not None and id(child) not in seen:
                    rec(child)

        rec(root)
        pents, bents, params, buffers, ps, bs = [], [], [], [], set(), set()
        for md in mods:  # Module.parameters() order: modules pre-order, then insertion order
            for name, t in md._parameters.items():
                pents.append((md, name, t))
                if t is not None and id(t) not in ps:
                    ps.add(id(t))
                    params.append(t)
        for md in mods:
            for name, t in md._buffers.items():
                bents.append((md, name, t))
                if t is not None and id(t) not in bs:
                    bs.add(id(t))
                    buffers.append(t)
        self.edges, self.pents, self.bents, self.params, self.buffers = edges, pents, bents, params, buffers
        self.mods = mods
        self.counts = [(m, len(m._modules), len(m._parameters), len(m._buffers)) for m in mods]

    def _valid(self, root):
        return (self.edges is not None and self.mods[0] is root
                and all(len(m._modules) == a and len(m._parameters) == b and len(m._buffers) == c
                        for m, a, b, c in self.counts)
                and all(m._modules[n] is c for m, n, c in self.edges)
                and all(m._parameters[n] is t for m, n, t in self.pents)
                and all(m._buffers[n] is t for m, n, t in self.bents))

    def get(self, root):
        if self.epoch == _STRUCT_EPOCH[0] and self.mods[0] is root:
            return self.params, self.buffers
        if not self._valid(root):
            self._walk(root)
        self.epoch = _STRUCT_EPOCH[0]
        return self.params, self.buffers


_DATA_PTR = torch.Tensor.data_ptr
_VERSION = operator.attrgetter("_version")


def _needs_grad(*ts):
    return torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


def _bn_modules(module):
    """The BatchNorm1d modules of ``module``'s tree; the walk (~1.4 ms on
    DSTDGCN) is cached on the module for the current structure epoch."""
    c = module.__dict__.get("_dstd_bn_cache")
    if c is not None and c[0] == _STRUCT_EPOCH[0]:
        return c[1]
    bns = [m for m in module.modules() if isinstance(m, nn.BatchNorm1d)]
    module.__dict__["_dstd_bn_cache"] = (_STRUCT_EPOCH[0], bns)
    return bns


def _bn_momentum(module):
    moms = {m.momentum for m in _bn_modules(module)}
    if len(moms) != 1 or None in moms:
        raise NotImplementedError(f"native train-mode BN needs one fixed momentum for every BatchNorm, got {moms}")
    return float(moms.pop())


def _count_batch(module, calls=1):
    """nn.BatchNorm1d bumps num_batches_tracked once per train forward
    (``calls``: a forward pair counts as two)."""
    t = [m.num_batches_tracked for m in _bn_modules(module) if m.num_batches_tracked is not None]
    if t:
        torch._foreach_add_(t, calls)


def _op_train_fwd_native(mod, mode, x, A, alpha):
    L = native.lib()
    B, cin, T, V = x.shape
    dev = x.device
    cout, red = mod.out_channels, mod.red_channels
    y = torch.empty(B, cout, T, V, dtype=torch.float32, device=dev)
    nbytes = L.dstd_dstdgc_train_saved_bytes_r(mode, B, cin, cout, T, V, red)
    saved = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    code = L.dstd_dstdgc_train_fwd_r(mode, native.ptr(x, "x"), B, cin, cout, T, V, red, native.gc_weights(mod),
                                     native.ptr(A, "A"), native.ptr(alpha, "alpha_m"), native.ptr(y, "y"),
                                     saved.data_ptr(), nbytes, native.stream_handle(dev))
    native.check(code, "dstd_dstdgc_train_fwd_r")
    return y, saved


class _OpTrain(torch.autograd.Function):
    """DSTDGC forward + native backward (reference :80-94 under autograd);
    both directions are torch.library ops (dstd::dstdgc_train_forward /
    dstdgc_train_backward, below)."""

    @staticmethod
    def forward(ctx, mod, mode, x, A, alpha, *params):
        y, saved = torch.ops.dstd.dstdgc_train_forward(x, A, alpha, list(params), mod._dstd_uid)
        ctx.mod, ctx.saved_buf = mod, saved
        ctx.params = list(params)
        ctx.save_for_backward(x, A, alpha)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, A, alpha = ctx.saved_tensors
        need_dx = bool(ctx.needs_input_grad[2])
        dx, dA, dalpha, flat = torch.ops.dstd.dstdgc_train_backward(x, A, alpha, ctx.saved_buf, dy.contiguous(),
                                                                    ctx.params, ctx.mod._dstd_uid, need_dx)
        ctx.saved_buf = None
        arena = native.GradArena(ctx.params, x.device, buf=flat)
        return (None, None, dx if need_dx else None, dA, dalpha, *arena.views())


def _bn_flags(module):
    """Batch statistics in train mode; the running statistics, not updated,
    under .eval() (an eval-mode forward that autograd differentiates)."""
    return 0 if module.training else native.TRAIN_RUNNING_STATS


def _block_train_fwd_native(blk, x, flags, momentum):
    L = native.lib()
    B, cin, T, V = x.shape
    dev = x.device
    y = torch.empty(B, blk.out_channels, T, V, dtype=torch.float32, device=dev)
    nbytes = L.dstd_block_train_saved_bytes(B, cin, blk.out_channels, T, V)
    saved = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    code = L.dstd_block_train_fwd_ex(native.block_struct(blk), native.ptr(x, "x"), B, T, V, momentum,
                                     native.ptr(y, "y"), saved.data_ptr(), nbytes, native.stream_handle(dev), flags)
    native.check(code, "dstd_block_train_fwd_ex")
    return y, saved


def _block_train_bwd_native(blk, x, saved, dy, flags, arena, need_dx):
    L = native.lib()
    B, cin, T, V = x.shape
    dev = x.device
    dx = torch.zeros_like(x) if need_dx else None
    ws = native.workspace(dev, L.dstd_block_train_workspace_bytes(B, cin, blk.out_channels, T, V))
    code = L.dstd_block_train_bwd_ex(native.block_struct(blk), native.ptr(x, "x"), B, T, V, saved.data_ptr(),
                                     saved.numel(), native.ptr(dy, "dy"), dx.data_ptr() if dx is not None else None,
                                     native.block_grads(blk, arena), ws.data_ptr(), ws.numel(),
                                     native.stream_handle(dev), flags)
    native.check(code, "dstd_block_train_bwd_ex")
    return dx


def _model_train_fwd_native(model, x, flags, momentum, drop, seed):
    L = native.lib()
    n, t, v, c = x.shape
    dev = x.device
    y = torch.empty_like(x)
    nbytes = L.dstd_model_train_saved_bytes(n, t, v, model.num_feature, model.num_layers)
    saved = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    args = (model._native_params(), native.ptr(x, "x"), n, momentum, drop, seed, native.ptr(y, "y"),
            saved.data_ptr(), nbytes, native.stream_handle(dev), flags)
    sync = _bn_sync(model, flags)
    if sync is not None:  # cross-rank BatchNorm (dstd_dist.convert_sync_batchnorm)
        native.check(L.dstd_model_train_fwd_sync(*args, sync), "dstd_model_train_fwd_sync")
    else:
        native.check(L.dstd_model_train_fwd_ex(*args), "dstd_model_train_fwd_ex")
    return y, saved


def _bn_sync(model, flags):
    """The model's dstd_bn_sync (dstd_dist.BnSync) when its BatchNorms run on
    batch statistics; None for per-rank BatchNorm or running statistics."""
    s = model.__dict__.get("_dstd_bn_sync")
    if s is None or flags & native.TRAIN_RUNNING_STATS:
        return None
    return s.struct_ref()


def _model_train_bwd_native(model, x, saved, dy, flags, drop, seed, g, need_dx):
    L = native.lib()
    n, t, v, c = x.shape
    dev = x.device
    ws = native.workspace(dev, L.dstd_model_train_workspace_bytes(n, t, v, model.num_feature, model.num_layers))
    dx = torch.empty_like(x) if need_dx else None
    args = (model._native_params(), native.ptr(x, "x"), n, drop, seed, saved.data_ptr(), saved.numel(),
            native.ptr(dy, "dy"), g, dx.data_ptr() if dx is not None else None, ws.data_ptr(), ws.numel(),
            native.stream_handle(dev), flags)
    sync = _bn_sync(model, flags)
    if sync is not None:
        native.check(L.dstd_model_train_bwd_sync(*args, sync), "dstd_model_train_bwd_sync")
    else:
        native.check(L.dstd_model_train_bwd_ex(*args), "dstd_model_train_bwd_ex")
    return dx


class _BlockTrain(torch.autograd.Function):
    """DSTDGCB forward + native backward (reference :141-163): train-mode BN,
    or running-statistics BN for an eval-mode block under autograd.  Both
    directions are torch.library ops (dstd::dstdgcb_train_forward /
    dstdgcb_train_backward, below) over the C ABI."""

    @staticmethod
    def forward(ctx, blk, x, *params):
        flags = _bn_flags(blk)
        y, saved = torch.ops.dstd.dstdgcb_train_forward(x, list(params), list(blk.buffers()), blk._dstd_uid, flags,
                                                        _bn_momentum(blk))
        if not flags:
            _count_batch(blk)
        ctx.blk, ctx.saved_buf, ctx.flags = blk, saved, flags
        ctx.params = list(params)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        need_dx = bool(ctx.needs_input_grad[1])
        dx, flat = torch.ops.dstd.dstdgcb_train_backward(x, ctx.saved_buf, dy.contiguous(), ctx.params,
                                                         ctx.blk._dstd_uid, ctx.flags, need_dx)
        ctx.saved_buf = None
        arena = native.GradArena(ctx.params, x.device, buf=flat)
        return (None, dx if need_dx else None, *arena.views())


@torch._dynamo.disable
def _host_seed(model):
    """A dropout seed for the op branch of _ModelTrain: an integer drawn on
    the host at run time (under torch.compile this is a graph break, not a
    traced random value -- dynamo would turn one into a tensor, which the ops'
    integer `seed` cannot take).  Taken from the model device's generator --
    the one the eager branch draws its device seed from -- as its (seed,
    philox offset) pair, whose offset it then advances as one device draw
    would: torch.manual_seed makes compiled training with dropout
    reproducible, compiled and eager steps consume the same stream, and the
    global CPU stream (samplers, DataLoader base seeds) is not touched
    (ADVICE r05)."""
    dev = next(model.parameters()).device
    g = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    seed, off = g.initial_seed(), g.get_offset()
    g.set_offset(off + 4)
    return (seed * 0x9E3779B97F4A7C15 + (off + 1) * 0xBF58476D1CE4E5B9) % (2 ** 62)


class _ModelTrain(torch.autograd.Function):
    """DSTDGCN forward + native backward (reference :293-317): train mode, or
    an eval-mode model under autograd (running-statistics BN, no dropout).
    Both directions are torch.library ops (dstd::dstdgcn_train_forward /
    dstdgcn_train_backward, below) over the C ABI; eager forwards call the
    forward op's implementation directly (as the eval forward does), and the
    opt-in in-place gradient arena calls the C ABI directly (it writes .grad
    as a side effect, which an op cannot)."""

    @staticmethod
    def forward(ctx, model, paired, x, *params):
        # paired: x is two train-mode batches of B/2 (DSTDGCN.forward_pair)
        flags = _bn_flags(model) | (native.TRAIN_PAIRED if paired else 0)
        if getattr(model, "_dstd_one_stream", False):  # the backward's launches all on the caller's stream
            flags |= native.TRAIN_ONE_STREAM
        drop = float(model.do_in.p) if model.do_in.training else 0.0
        seed, ctx.seed_t = 0, None
        eager = type(x) is torch.Tensor and not torch.compiler.is_compiling()
        if drop > 0 and eager:
            # the dropout seed is drawn on the device and read there
            # (DSTD_TRAIN_SEED_DEVICE): no host round trip, and a captured HIP
            # graph (engine.GraphedStep) draws a fresh mask per replay; the
            # tensor lives in ctx until the backward has regenerated the mask
            ctx.seed_t = torch.randint(0, 2 ** 62, (1,), device=x.device, dtype=torch.int64)
            seed = ctx.seed_t.data_ptr()
            flags |= native.TRAIN_SEED_DEVICE
        elif drop > 0:
            # the op branch (torch.compile, subclass inputs): the ops' schema
            # carries the seed as an integer, so it is drawn on the host -- a
            # device tensor read by pointer would be invisible to the tracer
            # (and a FakeTensor has no data pointer).  Drawn outside the traced
            # region (_host_seed), so it stays an integer and every compiled call
            # gets a new mask
            seed = _host_seed(model)
        buffers = model._tree.get(model)[1]
        if eager:
            # eager: the op's implementation without the dispatcher's boxing
            # of ~300 tensor arguments (~0.3 ms of host time per step); the
            # running statistics it updates get the version bump the op's
            # mutates_args declares (the eval forward's constant cache keys
            # on versions)
            y, saved = _model_train_fwd_native(model, x, flags, _bn_momentum(model), drop, seed)
            if not flags & native.TRAIN_RUNNING_STATS:
                torch.autograd.graph.increment_version(buffers)
        else:
            y, saved = torch.ops.dstd.dstdgcn_train_forward(x, list(params), buffers, model._dstd_uid,
                                                            flags, _bn_momentum(model), drop, seed)
        if not flags & native.TRAIN_RUNNING_STATS:
            _count_batch(model, 2 if paired else 1)
        ctx.model, ctx.saved_buf, ctx.drop, ctx.seed, ctx.flags = model, saved, drop, seed, flags
        # anchored (_anchor_of): the parameters are not the Function's inputs
        ctx.anchored = len(params) == 1 and params[0] is getattr(model, "_dstd_anchor_t", None)
        # the backward reuses them (a module walk costs ~0.7 ms)
        ctx.params = model._tree.get(model)[0] if ctx.anchored else list(params)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        model = ctx.model
        dev = x.device
        dy = dy.contiguous()
        need_dx = bool(ctx.needs_input_grad[2])
        # gradients accumulate straight into the parameters' .grad (one arena,
        # native +=) when the caller opted in (engine.PredictionEngine.train
        # sets model._dstd_inplace_grads) and no parameter carries hooks; else
        # the backward op fills a fresh arena whose views autograd accumulates
        # (hooks, DDP and torch.autograd.grad see ordinary gradients)
        if ctx.anchored or (getattr(model, "_dstd_inplace_grads", False) and not any(
                p._backward_hooks or getattr(p, "_post_accumulate_grad_hooks", None) for p in ctx.params)):
            arena, direct = native.grad_sink(model, ctx.params, dev)
            if direct:
                g = getattr(arena, "model_grads", None)
                if g is None:  # the persistent arena: its pointer table is reused
                    g = arena.model_grads = model._native_grads(arena)
                dx = _model_train_bwd_native(model, x, ctx.saved_buf, dy, ctx.flags, ctx.drop, ctx.seed, g, need_dx)
                ctx.saved_buf = ctx.seed_t = None
                return (None, None, dx, *([None] * (1 if ctx.anchored else len(arena.params))))
        dx, flat = torch.ops.dstd.dstdgcn_train_backward(x, ctx.saved_buf, dy, ctx.params, model._dstd_uid, ctx.flags,
                                                         ctx.drop, ctx.seed, need_dx)
        ctx.saved_buf = ctx.seed_t = None
        arena = native.GradArena(ctx.params, dev, buf=flat)
        if ctx.anchored:
            # .grad was set by someone else since the forward: accumulate as
            # autograd's AccumulateGrad would (no hooks: _anchor_of checked)
            for p, v in zip(arena.params, arena.views()):
                if v is not None and p.requires_grad:
                    if p.grad is None:
                        p.grad = v.clone()
                    else:
                        p.grad.add_(v)
            return (None, None, dx if need_dx else None, None)
        return (None, None, dx if need_dx else None, *arena.views())


def _anchor_of(model, x, params):
    """The Function's parameter inputs for a train-mode call: ``params``, or
    -- in the opt-in in-place gradient mode (model._dstd_inplace_grads, set by
    engine.PredictionEngine.train), eager, no parameter hooks -- one empty
    leaf that requires grad standing in for all of them.  The backward writes
    the parameters' .grad itself in that mode (native.grad_sink) and returns
    None for each of them, so autograd needs no edge per parameter: ~300
    inputs cost the host ~1 ms per step in Function.apply and the engine's
    walk of the backward graph (measured on this container's CPU: 1.9 ms
    against 0.1 ms for a 2-output Function with 300 vs 1 input)."""
    if not (getattr(model, "_dstd_inplace_grads", False) and torch.is_grad_enabled()
            and type(x) is torch.Tensor and not torch.compiler.is_compiling()):
        return params
    if not any(p.requires_grad for p in params) or any(
            p._backward_hooks or getattr(p, "_post_accumulate_grad_hooks", None) for p in params):
        return params
    a = getattr(model, "_dstd_anchor_t", None)
    if a is None:
        a = model._dstd_anchor_t = torch.empty(0, requires_grad=True)
    return [a]


class _ModelTrainPair(torch.autograd.Function):
    """DSTDGCN.forward_pair's Function: _ModelTrain over the concatenated
    pair (DSTD_TRAIN_PAIRED) with the two halves as two outputs.  The backward
    joins their gradients with one copy; slicing one output instead left it to
    autograd's slice backward -- a zero-filled pair-sized buffer and a copy per
    half, then their sum (five launches and their host time per step)."""

    @staticmethod
    def forward(ctx, model, n, x, *params):
        y = _ModelTrain.forward(ctx, model, True, x, *params)
        return y[:n], y[n:]

    @staticmethod
    def backward(ctx, d1, d2):
        (x,) = ctx.saved_tensors
        n = x.shape[0] // 2
        if d1 is None:
            d1 = x.new_zeros((n,) + tuple(x.shape[1:]))
        if d2 is None:
            d2 = x.new_zeros((x.shape[0] - n,) + tuple(x.shape[1:]))
        # (argument positions: model, n, x, params -- as _ModelTrain's model, paired, x, params)
        return _ModelTrain.backward(ctx, torch.cat([d1, d2]))


class BatchNorm(nn.Module):
    """BN1d over C*V channels of an NCTV tensor (reference :35-50).  Glue only:
    on the hot path every BatchNorm is folded into a kernel epilogue."""

    def __init__(self, feature_channels, joint_dim, time_dim):
        super().__init__()
        self.c = feature_channels
        self.v = joint_dim
        self.t = time_dim
        self.bn = nn.BatchNorm1d(feature_channels * joint_dim)

    def forward(self, x):
        n, c, t, v = x.shape
        assert (c, t, v) == (self.c, self.t, self.v)
        y = self.bn(x.transpose(2, 3).reshape(n, c * v, t))
        return y.reshape(n, c, v, t).transpose(2, 3).contiguous()


class DSTDGC(_NativeModule):
    """Dynamic graph convolution (reference :53-94); ``mode`` spatial or temporal."""

    def __init__(self, in_channels, out_channels, ref_channels, kpt_channels, red_channels=2, mode="spatial"):
        super().__init__()
        if mode not in ("spatial", "temporal"):
            raise AssertionError(f"mode must be spatial or temporal, got {mode}")
        if not 1 <= red_channels <= 8:
            raise NotImplementedError(f"red_channels={red_channels}: this build covers 1..8 (every shipped config uses 2)")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.ref_channels = ref_channels
        self.kpt_channels = kpt_channels
        self.red_channels = red_channels
        self.mode = mode
        self.conv_m1 = nn.Conv2d(in_channels, red_channels, 1)
        self.conv_m2 = nn.Conv2d(in_channels, red_channels, 1)
        self.conv_rm = nn.Conv2d(red_channels * ref_channels, ref_channels, 1)
        self.tanh = nn.Tanh()
        self.conv_f = nn.Conv2d(in_channels, out_channels, 1)
        self.init_parameter()
        _register(self)

    def init_parameter(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                conv_init(m)

    def forward(self, x, A=None, alpha_m=1):
        L = native.lib()
        B, cin, T, V = x.shape
        if cin != self.in_channels:
            raise ValueError(f"DSTDGC: expected {self.in_channels} input channels, got {cin}")
        x = x.contiguous()
        native.require_device(x, "x")
        dev = x.device
        if B == 0:  # empty batch: empty output, as the reference's torch ops give
            return _mark(x.new_empty(0, self.out_channels, T, V), x)
        A = A.reshape(A.shape[-2], A.shape[-1]).contiguous()
        if not torch.is_tensor(alpha_m):
            alpha_m = torch.full((1,), float(alpha_m), dtype=torch.float32, device=dev)
        alpha = alpha_m.reshape(1).contiguous()
        mode = native.MODE_SPATIAL if self.mode == "spatial" else native.MODE_TEMPORAL
        params = list(self.parameters())
        if _needs_grad(x, A, alpha, *params):
            return _OpTrain.apply(self, mode, x, A, alpha, *params)
        return torch.ops.dstd.dstdgc_forward(x, A, alpha, params, self._dstd_uid)

    def _eval_native(self, x, A, alpha):
        """dstd_dstdgc_fwd on prepared operands (torch.ops.dstd.dstdgc_forward)."""
        L = native.lib()
        B, cin, T, V = x.shape
        dev = x.device
        mode = native.MODE_SPATIAL if self.mode == "spatial" else native.MODE_TEMPORAL
        if self.red_channels != 2:
            # the inference kernels carry exactly two P / Q channels; any other
            # red_channels runs the training forward (generic in it, exact fp32,
            # and the same function: DSTDGC has no BN or dropout)
            return _op_train_fwd_native(self, mode, x, A, alpha)[0]
        y = torch.empty(B, self.out_channels, T, V, dtype=torch.float32, device=dev)
        nbytes = L.dstd_dstdgc_workspace_bytes(mode, B, cin, self.out_channels, T, V)
        ws = native.workspace(dev, nbytes)
        w = native.gc_weights(self)
        code = L.dstd_dstdgc_fwd(mode, native.ptr(x, "x"), B, cin, self.out_channels, T, V, w,
                                 native.ptr(A, "A"), native.ptr(alpha, "alpha_m"), native.ptr(y, "y"),
                                 ws.data_ptr(), ws.numel(), native.stream_handle(dev))
        native.check(code, "dstd_dstdgc_fwd")
        return y


class DSTDGCB(_NativeModule):
    """DSTD-GC block: two spatial DSTDGCs on the skeleton priors, BN + residual
    + PReLU, one temporal DSTDGC (reference :97-163)."""

    def __init__(self, in_channels, out_channels, time_dim, joint_dim, layout="h36m"):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        A_s = Graph(layout).get_all_adjacency()
        A_t = Time(time_dim).get_all_adjacency()
        # registration order and the A_s/R_s alias follow the reference (:107-112)
        self.A_s = nn.Parameter(torch.tensor(A_s, dtype=torch.float32), False)
        self.W_s = nn.Parameter(torch.zeros_like(self.A_s))
        self.R_s = nn.Parameter(self.A_s.data)  # same storage as A_s
        self.A_t = nn.Parameter(torch.tensor(A_t, dtype=torch.float32), False)
        self.R_t = nn.Parameter(torch.zeros_like(self.A_t))
        self.conv_s = nn.ModuleList()
        self.conv_t = nn.ModuleList()
        if in_channels != out_channels:
            self.residual = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1),
                                          BatchNorm(out_channels, joint_dim, time_dim))
        else:
            self.residual = lambda x: x
        for _ in range(A_s.shape[0]):
            self.conv_s.append(DSTDGC(in_channels, out_channels, time_dim, joint_dim, mode="spatial"))
        self.alpha_sm = nn.Parameter(torch.zeros(1))
        self.bn = BatchNorm(out_channels, joint_dim, time_dim)
        for _ in range(A_t.shape[0]):
            self.conv_t.append(DSTDGC(out_channels, out_channels, joint_dim, time_dim, mode="temporal"))
        self.alpha_tm = nn.Parameter(torch.zeros(1))
        self.prelu = nn.PReLU()
        self.do = nn.Dropout(0.1)  # constructed but never applied (reference :133)
        # arithmetic of the eval forward's graph convolutions, per call
        # (include/dstd_gcn.h DSTD_FWD_EXACT_FP32): "split" or "fp32"
        self.gc_arithmetic = "split"
        _register(self)

    def init_parameter(self):
        stdt = 1.0 / math.sqrt(self.R_t.size(1))
        self.R_t.data.uniform_(-stdt, stdt)
        stdt = 1.0 / math.sqrt(self.R_s.size(1))
        self.R_s.data.uniform_(-stdt, stdt)

    def forward(self, x):
        L = native.lib()
        B, cin, T, V = x.shape
        x = x.contiguous()
        native.require_device(x, "x")
        if B == 0 and not self.training:  # empty batch: empty output (reference torch semantics)
            return _mark(x.new_empty(0, self.out_channels, T, V), x, *self.parameters())
        params = list(self.parameters())
        if self.training or _needs_grad(x, *params):
            # train mode, or an eval-mode output autograd differentiates: the
            # native training path (running-statistics BN in eval mode)
            return _BlockTrain.apply(self, x, *params)
        tensors = params + list(self.buffers())
        # _dstd_fwd_flags: extra per-call schedule flags (tests / A-B: include/dstd_gcn.h DSTD_FWD_*)
        return torch.ops.dstd.dstdgcb_forward(x, tensors, self._dstd_uid, self.out_channels,
                                              native.arith_flags(self.gc_arithmetic) | self._dstd_fwd_flags)

    def _eval_native(self, x, flags):
        """dstd_block_fwd_ex (torch.ops.dstd.dstdgcb_forward)."""
        L = native.lib()
        B, cin, T, V = x.shape
        dev = x.device
        y = torch.empty(B, self.out_channels, T, V, dtype=torch.float32, device=dev)
        nbytes = L.dstd_block_workspace_bytes(B, cin, self.out_channels, T, V)
        ws = native.workspace(dev, nbytes)
        p = native.block_struct(self)
        code = L.dstd_block_fwd_ex(p, native.ptr(x, "x"), B, T, V, native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                                   native.stream_handle(dev), flags)
        native.check(code, "dstd_block_fwd_ex")
        return y


def _ptr_or_none(t):
    return t.data_ptr() if t is not None else None


class _CTGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Tm, A, A_fixed):
        L = native.lib()
        B, C, T, V = x.shape
        dev = x.device
        y = torch.empty_like(x)
        ws = native.workspace(dev, L.dstd_ctg_workspace_bytes(B, C, T, V))
        code = L.dstd_ctg_fwd(native.ptr(x, "x"), B, C, T, V, native.ptr(Tm, "T"), native.ptr(A, "A"),
                              native.ptr(A_fixed, "A_fixed"), native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                              native.stream_handle(dev))
        native.check(code, "dstd_ctg_fwd")
        ctx.save_for_backward(x, Tm, A, A_fixed)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = native.lib()
        x, Tm, A, A_fixed = ctx.saved_tensors
        B, C, T, V = x.shape
        dev = x.device
        dy = dy.contiguous()
        dx = torch.zeros_like(x) if ctx.needs_input_grad[0] else None
        dTm, dA = torch.zeros_like(Tm), torch.zeros_like(A)
        ws = native.workspace(dev, L.dstd_ctg_workspace_bytes(B, C, T, V))
        code = L.dstd_ctg_bwd(native.ptr(x, "x"), B, C, T, V, native.ptr(Tm, "T"), native.ptr(A, "A"),
                              native.ptr(A_fixed, "A_fixed"), native.ptr(dy, "dy"), _ptr_or_none(dx), dTm.data_ptr(),
                              dA.data_ptr(), ws.data_ptr(), ws.numel(), native.stream_handle(dev))
        native.check(code, "dstd_ctg_bwd")
        return dx, dTm, dA, None


class ConvTemporalGraphical(nn.Module):
    """Learnable temporal (T [V,T,T]) then spatial (A [T,V,V] + fixed skeleton)
    graph mixing (reference :166-188).  Only reachable through
    ST_GCNN_layer(refine=False), which no shipped config builds."""

    def __init__(self, time_dim, joints_dim, layout="h36m"):
        super().__init__()
        self.A = nn.Parameter(torch.FloatTensor(time_dim, joints_dim, joints_dim))
        stdv = 1.0 / math.sqrt(self.A.size(1))
        self.A.data.uniform_(-stdv, stdv)
        self.T = nn.Parameter(torch.FloatTensor(joints_dim, time_dim, time_dim))
        stdv = 1.0 / math.sqrt(self.T.size(1))
        self.T.data.uniform_(-stdv, stdv)
        adj = Graph(layout).get_adjacency()[np.newaxis, :]
        self.A_fixed = nn.Parameter(torch.FloatTensor(adj), requires_grad=False)

    def forward(self, x):
        x = x.contiguous()
        native.require_device(x, "x")
        return _CTGFn.apply(x, self.T.contiguous(), self.A.contiguous(), self.A_fixed.contiguous())


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, geom):
        L = native.lib()
        B, cin, H, W = x.shape
        cout, kh, kw, sh, sw, ph, pw = geom
        Ho, Wo = (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1
        dev = x.device
        y = torch.empty(B, cout, Ho, Wo, dtype=torch.float32, device=dev)
        nbytes = L.dstd_conv2d_workspace_bytes(B, cin, cout, H, W, kh, kw, sh, sw, ph, pw)
        ws = native.workspace(dev, nbytes)
        code = L.dstd_conv2d_fwd(native.ptr(x, "x"), B, cin, H, W, native.ptr(weight, "weight"), _ptr_or_none(bias),
                                 cout, kh, kw, sh, sw, ph, pw, native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                                 native.stream_handle(dev))
        native.check(code, "dstd_conv2d_fwd")
        ctx.geom = geom
        ctx.save_for_backward(x, weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = native.lib()
        x, weight, bias = ctx.saved_tensors
        B, cin, H, W = x.shape
        cout, kh, kw, sh, sw, ph, pw = ctx.geom
        dev = x.device
        dy = dy.contiguous()
        dx = torch.zeros_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.zeros_like(weight)
        db = torch.zeros_like(bias) if bias is not None else None
        nbytes = L.dstd_conv2d_workspace_bytes(B, cin, cout, H, W, kh, kw, sh, sw, ph, pw)
        ws = native.workspace(dev, nbytes)
        code = L.dstd_conv2d_bwd(native.ptr(x, "x"), B, cin, H, W, native.ptr(weight, "weight"), cout, kh, kw, sh, sw,
                                 ph, pw, native.ptr(dy, "dy"), _ptr_or_none(dx), dw.data_ptr(), _ptr_or_none(db),
                                 ws.data_ptr(), ws.numel(), native.stream_handle(dev))
        native.check(code, "dstd_conv2d_bwd")
        return dx, dw, db, None


class Conv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state_dict) computed by the native kernels
    (include/dstd_gcn_aux.h); groups = dilation = 1, zero padding."""

    def forward(self, x):
        if self.groups != 1 or self.dilation != (1, 1) or self.padding_mode != "zeros" or isinstance(self.padding,
                                                                                                       str):
            raise NotImplementedError("native Conv2d: groups=1, dilation=1, numeric zero padding only")
        x = x.contiguous()
        native.require_device(x, "x")
        geom = (self.out_channels, *self.kernel_size, *self.stride, *self.padding)
        return _Conv2dFn.apply(x, self.weight.contiguous(), None if self.bias is None else self.bias.contiguous(),
                               geom)


class ST_GCNN_layer(nn.Module):
    """Wrapper of one DSTDGCB plus an optional residual (reference :191-249).
    Every shipped config builds ``refine=True``; the STS-GCN style
    ``refine=False`` branch (ConvTemporalGraphical + a k_t x k_v Conv2d,
    :218-223) runs on the native kernels of include/dstd_gcn_aux.h."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, time_dim, joints_dim, bias=True,
                 refine=False, residual=True, layout="h36m"):
        super().__init__()
        self.kernel_size = kernel_size
        self.refine = refine
        assert self.kernel_size[0] % 2 == 1
        assert self.kernel_size[1] % 2 == 1
        padding = ((self.kernel_size[0] - 1) // 2, (self.kernel_size[1] - 1) // 2)
        if refine:
            self.stgcn = nn.ModuleList(
                [nn.Sequential(DSTDGCB(in_channels, out_channels, time_dim, joints_dim, layout))])
        else:
            self.stgcn = nn.Sequential(ConvTemporalGraphical(time_dim, joints_dim, layout),
                                       Conv2d(in_channels, out_channels, (self.kernel_size[0], self.kernel_size[1]),
                                              (stride, stride), padding))
        if not residual:
            self.residual = None
        elif stride != 1 or in_channels != out_channels:
            self.residual = Conv2d(in_channels, out_channels, kernel_size=1, stride=1)
        else:
            self.residual = nn.Identity()
        self.apply(weights_init)

    def forward(self, x):
        if self.refine:
            y = None
            for stb in self.stgcn:
                z = stb(x)
                y = z if y is None else y + z
        else:
            y = self.stgcn(x)
        if self.residual is not None:
            y = y + self.residual(x)
        return y


class DSTDGCN(_NativeModule):
    """The whole network (reference :252-317)."""

    def __init__(self, input_channels, input_time_frame, output_time_frame, st_gcnn_dropout, joints_to_consider,
                 num_feature=64, num_layers=7, layout="h36m"):
        super().__init__()
        self.input_time_frame = input_time_frame
        self.output_time_frame = output_time_frame
        self.joints_to_consider = joints_to_consider
        self.input_channels = input_channels
        self.num_feature = num_feature
        self.num_layers = num_layers
        self.encoders = nn.ModuleList()
        T = input_time_frame + output_time_frame
        self.conv_st_in = ST_GCNN_layer(input_channels, num_feature, [1, 1], 1, T, joints_to_consider, True, True,
                                        False, layout)
        self.bn_in = BatchNorm(num_feature, joints_to_consider, T)
        self.do_in = nn.Dropout(st_gcnn_dropout)
        for _ in range(num_layers):
            self.encoders.append(
                nn.Sequential(ST_GCNN_layer(num_feature, num_feature, [1, 1], 1, T, joints_to_consider, False, True,
                                            True, layout),
                              BatchNorm(num_feature, joints_to_consider, T),
                              nn.PReLU()))
        self.conv_st_out = ST_GCNN_layer(num_feature, input_channels // 2, [1, 1], 1, T, joints_to_consider, True,
                                         True, False, layout)
        self.prelu = nn.PReLU()
        self._native = None
        self._tree = _TensorTree()
        self.gc_arithmetic = "split"  # see DSTDGCB; set_gc_arithmetic() sets the whole tree
        self._dstd_gen = 0
        _register(self)
        self.register_load_state_dict_post_hook(lambda mod, incompatible: invalidate_native_cache(mod))

    def set_gc_arithmetic(self, mode):
        """"split" (default) or "fp32" for this model's eval forward and every
        DSTDGCB in it (include/dstd_gcn.h DSTD_FWD_EXACT_FP32)."""
        native.arith_flags(mode)  # validates
        for m in self.modules():
            if isinstance(m, (DSTDGCN, DSTDGCB)):
                m.gc_arithmetic = mode
        return self

    # -- native parameter block ---------------------------------------------
    def _native_params(self):
        params, buffers = self._tree.get(self)
        if self._native is not None and self._native[2] is params:
            tensors = self._native_tensors
        else:
            tensors = self._native_tensors = params + buffers
        ptrs = tuple(map(_DATA_PTR, tensors))
        if self._native is not None and self._native[0] == ptrs:
            return self._native[1]
        p = native.ModelParams()
        p.T = self.input_time_frame + self.output_time_frame
        p.V = self.joints_to_consider
        p.num_layers = self.num_layers
        p.num_feature = self.num_feature
        p.in_channels = self.input_channels
        if self.num_layers > native.MAX_LAYERS:
            raise ValueError(f"num_layers {self.num_layers} > {native.MAX_LAYERS}")
        p.st_in = native.block_struct(self.conv_st_in.stgcn[0][0])
        p.bn_in = native.bn_struct(self.bn_in)
        p.prelu = native.ptr(self.prelu.weight, "prelu.weight")
        for i, enc in enumerate(self.encoders):
            p.enc[i] = native.block_struct(enc[0].stgcn[0][0])
            p.enc_bn[i] = native.bn_struct(enc[1])
            p.enc_prelu[i] = native.ptr(enc[2].weight, f"encoders.{i}.2.weight")
        p.st_out = native.block_struct(self.conv_st_out.stgcn[0][0])
        self._native = (ptrs, p, params)
        return p

    def _native_grads(self, arena):
        g = native.ModelGrads()
        g.st_in = native.block_grads(self.conv_st_in.stgcn[0][0], arena)
        g.bn_in = native.bn_grads(self.bn_in, arena)
        g.prelu = arena.ptr(self.prelu.weight)
        for i, enc in enumerate(self.encoders):
            g.enc[i] = native.block_grads(enc[0].stgcn[0][0], arena)
            g.enc_bn[i] = native.bn_grads(enc[1], arena)
            g.enc_prelu[i] = arena.ptr(enc[2].weight)
        g.st_out = native.block_grads(self.conv_st_out.stgcn[0][0], arena)
        return g

    def forward(self, x):
        n, t, v, c = x.shape
        assert t == self.input_time_frame + self.output_time_frame
        if c != self.input_channels // 2 or v != self.joints_to_consider:
            raise ValueError(f"DSTDGCN: expected [N, {t}, {self.joints_to_consider}, {self.input_channels // 2}], "
                             f"got {list(x.shape)}")
        L = native.lib()
        x = x.contiguous()
        native.require_device(x, "x")
        if n == 0 and not self.training:  # empty batch: empty output (reference torch semantics)
            return _mark(torch.empty_like(x), x, *self._tree.get(self)[0])
        params, buffers = self._tree.get(self)
        if self.training or _needs_grad(x, *params):
            # train mode, or an eval-mode forward autograd differentiates (the
            # reference back-propagates through running-statistics BN there)
            return _ModelTrain.apply(self, False, x, *_anchor_of(self, x, params))
        flags = native.arith_flags(self.gc_arithmetic)
        if type(x) is not torch.Tensor or torch.compiler.is_compiling():
            # tracing (torch.compile, FakeTensor): the custom op, whose inputs
            # name every tensor the forward reads
            return torch.ops.dstd.dstdgcn_forward(x, params + buffers, self._dstd_uid, flags)
        # eager: the op's implementation without the dispatcher's per-call
        # boxing of ~400 tensor arguments
        y = torch.empty_like(x)
        self._forward_native(x, y, arith=flags)
        return y

    def forward_pair(self, x1, x2):
        """``(self(x1), self(x2))`` -- PredictionEngine.train's forward of a
        batch and of its time reversal (engine/prediction.py:231-287) -- as
        ONE native launch sequence over the concatenated batch.  In train mode
        every BatchNorm keeps each half's own batch statistics and the running
        statistics take x1's update then x2's (DSTD_TRAIN_PAIRED), so outputs,
        gradients and buffers are those of the two calls; elsewhere (eval, or
        shapes that differ) it is the two calls."""
        if not self.training or x1.shape != x2.shape or x1.shape[0] == 0 or x1.device != x2.device:
            return self(x1), self(x2)
        n, t, v, c = x1.shape
        assert t == self.input_time_frame + self.output_time_frame
        if c != self.input_channels // 2 or v != self.joints_to_consider:
            raise ValueError(f"DSTDGCN: expected [N, {t}, {self.joints_to_consider}, {self.input_channels // 2}], "
                             f"got {list(x1.shape)}")
        native.lib()
        x = torch.cat([x1, x2]).contiguous()
        native.require_device(x, "x")
        params = self._tree.get(self)[0]
        return _ModelTrainPair.apply(self, n, x, *_anchor_of(self, x, params))

    def graphed(self, x, frozen=False):
        """The eval forward for inputs shaped like ``x`` captured once into a
        HIP graph (no per-call launch or Python cost at small
        batch).  Returns ``run(x_new) -> y``: copies ``x_new`` into the graph's
        static input (skipped when it is that tensor, ``run.input``), replays
        the forward's launches and returns the graph's static output
        ``run.output`` (overwritten by the next replay).  By default every
        replay also re-runs the two launches that fold BatchNorm and prepare
        the split weight images, so in-place parameter updates are seen by the
        next replay.  ``frozen=True`` (serving fixed weights): the first call
        folds, later ones replay the GC launches alone; after an in-place
        parameter update call ``run.refresh()``.  New parameter storage (e.g.
        ``load_state_dict`` into fresh tensors, ``.to()``) needs a new capture."""
        if self.training:
            raise RuntimeError("DSTDGCN.graphed captures the eval forward: call .eval() first")
        dev = x.device
        native.require_device(x, "x")
        x_static = x.detach().clone().contiguous()
        y_static = torch.empty_like(x_static)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(2):  # library load, per-kernel attributes, workspace
                self(x_static)
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)  # a stream of its own: its workspace is private to this graph
        with torch.no_grad(), torch.cuda.graph(g, stream=cap):
            self._forward_native(x_static, y_static)
        gf = None
        if frozen:
            # the same forward again on the same workspace: the claim finds the
            # constants graph g folds there (same tag), so this capture holds
            # only the GC launches
            gf = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(gf, stream=cap):
                self._forward_native(x_static, y_static)
        # the capture's workspace lives in the graph's memory pool: keep it
        # with the graph and out of the eager cache
        ws = native._ws_cache.pop((str(dev), cap.cuda_stream), (None, None))[0]
        state = {"folded": False}

        def run(x_new):
            if x_new is not x_static:
                x_static.copy_(x_new)
            if gf is not None and state["folded"]:
                gf.replay()
            else:
                g.replay()
                state["folded"] = True
            return y_static

        def refresh():
            """(frozen) parameters changed in place: the next call refolds."""
            state["folded"] = False

        run.graph, run.graph_frozen, run.input, run.output, run._workspace = g, gf, x_static, y_static, ws
        run.refresh = refresh
        return run

    def _forward_native(self, x, y, prof=None, arith=None):
        """One eval forward through dstd_model_fwd_ex.  The folded constants
        and split-f16 weight images a forward leaves in the workspace are
        reused when nothing changed since: same model instance (a token never
        reused) and cache generation (invalidate_native_cache), same parameter
        storage, torch version counters unchanged (no in-place update), batch
        size, arithmetic, and no other user of the workspace in between.
        Tensors without version counters (inference tensors) never reuse."""
        L = native.lib()
        n, t, v, _ = x.shape
        dev = x.device
        if prof is None:  # event brackets requested through the module (bench.py probes model(x) itself)
            prof = getattr(self, "_dstd_profile", None)
        p = self._native_params()
        flags = (native.arith_flags(self.gc_arithmetic) if arith is None else arith) | self._dstd_fwd_flags
        try:
            versions = tuple(map(_VERSION, self._native_tensors))
            tag = (self._dstd_uid, self._dstd_gen, self._native[0], n, flags, versions)
        except RuntimeError:  # "Inference tensors do not track version counter"
            tag = None
        nbytes = L.dstd_model_workspace_bytes(n, t, v, self.num_feature, self.num_layers)
        ws, reuse = native.workspace_claim(dev, nbytes, tag)
        if reuse:
            flags |= native.FWD_REUSE_CONSTANTS
        code = L.dstd_model_fwd_ex(p, native.ptr(x, "x"), n, native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                                   native.stream_handle(dev), flags, prof)
        native.check(code, "dstd_model_fwd_ex")


# ---------------------------------------------------------------------------
# torch.library ops: the eval forwards as custom operators with
# fake (meta) kernels, so torch.compile / FakeTensor tracing see them as single
# ops with known output shapes.  Each op receives every tensor of its module
# (the data dependencies) plus the module's instance token, under which the
# implementation finds the module that lays out the C parameter struct
# (include/dstd_gcn.h); underneath is the same C ABI call as before.
# ---------------------------------------------------------------------------
def _instance(uid):
    mod = _INSTANCES.get(uid)
    if mod is None:
        raise RuntimeError(f"dstd op: no live DSTD module with instance token {uid}")
    return mod


@torch.library.custom_op("dstd::dstdgc_forward", mutates_args=())
def _op_dstdgc_forward(x: torch.Tensor, A: torch.Tensor, alpha: torch.Tensor, weights: List[torch.Tensor],
                       uid: int) -> torch.Tensor:
    """DSTDGC.forward eval (reference :80-94) -> dstd_dstdgc_fwd."""
    return _instance(uid)._eval_native(x, A, alpha)


@_op_dstdgc_forward.register_fake
def _(x, A, alpha, weights, uid):
    # weights in DSTDGC.parameters() order: conv_m1, conv_m2, conv_rm, conv_f (weight, bias)
    return x.new_empty(x.shape[0], weights[6].shape[0], x.shape[2], x.shape[3])


@torch.library.custom_op("dstd::dstdgcb_forward", mutates_args=())
def _op_dstdgcb_forward(x: torch.Tensor, tensors: List[torch.Tensor], uid: int, cout: int,
                        flags: int) -> torch.Tensor:
    """DSTDGCB.forward eval (reference :141-163) -> dstd_block_fwd_ex."""
    return _instance(uid)._eval_native(x, flags)


@_op_dstdgcb_forward.register_fake
def _(x, tensors, uid, cout, flags):
    return x.new_empty(x.shape[0], cout, x.shape[2], x.shape[3])


@torch.library.custom_op("dstd::dstdgcn_forward", mutates_args=())
def _op_dstdgcn_forward(x: torch.Tensor, tensors: List[torch.Tensor], uid: int, flags: int) -> torch.Tensor:
    """DSTDGCN.forward eval (reference :293-317) -> dstd_model_fwd_ex."""
    y = torch.empty_like(x)
    _instance(uid)._forward_native(x, y, arith=flags)
    return y


@_op_dstdgcn_forward.register_fake
def _(x, tensors, uid, flags):
    return torch.empty_like(x)


# Training directions: forward ops return the
# output and the saved-state buffer the backward op consumes; backward ops
# return the input gradient (empty when not needed) and every parameter
# gradient in one flat arena (dstd_native.GradArena layout, in params order).
# The forward ops update the BN running statistics among `buffers` in train
# mode (declared mutated).
@torch.library.custom_op("dstd::dstdgcb_train_forward", mutates_args=("buffers",))
def _op_dstdgcb_train_forward(x: torch.Tensor, params: List[torch.Tensor], buffers: List[torch.Tensor], uid: int,
                              flags: int, momentum: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """DSTDGCB forward with train-mode (or running-stats) BN -> dstd_block_train_fwd_ex."""
    return _block_train_fwd_native(_instance(uid), x, flags, momentum)


@_op_dstdgcb_train_forward.register_fake
def _(x, params, buffers, uid, flags, momentum):
    blk = _instance(uid)
    B, cin, T, V = x.shape
    nbytes = native.lib().dstd_block_train_saved_bytes(B, cin, blk.out_channels, T, V)
    return x.new_empty(B, blk.out_channels, T, V), x.new_empty(nbytes, dtype=torch.uint8)


@torch.library.custom_op("dstd::dstdgcb_train_backward", mutates_args=())
def _op_dstdgcb_train_backward(x: torch.Tensor, saved: torch.Tensor, dy: torch.Tensor, params: List[torch.Tensor],
                               uid: int, flags: int, need_dx: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """DSTDGCB backward -> dstd_block_train_bwd_ex."""
    blk = _instance(uid)
    # the arena is laid out over the module's own parameters (the native
    # pointer table resolves them by identity); `params` -- the same tensors
    # in normal use, copies under opcheck -- match them slot for slot
    arena = native.GradArena(list(blk.parameters()), x.device)
    dx = _block_train_bwd_native(blk, x, saved, dy, flags, arena, need_dx)
    return (dx if dx is not None else x.new_empty(0)), arena.buf


@_op_dstdgcb_train_backward.register_fake
def _(x, saved, dy, params, uid, flags, need_dx):
    return (torch.empty_like(x) if need_dx else x.new_empty(0)), x.new_empty(native.arena_numel(params))


@torch.library.custom_op("dstd::dstdgcn_train_forward", mutates_args=("buffers",))
def _op_dstdgcn_train_forward(x: torch.Tensor, params: List[torch.Tensor], buffers: List[torch.Tensor], uid: int,
                              flags: int, momentum: float, drop: float, seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """DSTDGCN forward with train-mode (or running-stats) BN -> dstd_model_train_fwd_ex."""
    return _model_train_fwd_native(_instance(uid), x, flags, momentum, drop, seed)


@_op_dstdgcn_train_forward.register_fake
def _(x, params, buffers, uid, flags, momentum, drop, seed):
    m = _instance(uid)
    n, t, v, c = x.shape
    nbytes = native.lib().dstd_model_train_saved_bytes(n, t, v, m.num_feature, m.num_layers)
    return torch.empty_like(x), x.new_empty(nbytes, dtype=torch.uint8)


@torch.library.custom_op("dstd::dstdgcn_train_backward", mutates_args=())
def _op_dstdgcn_train_backward(x: torch.Tensor, saved: torch.Tensor, dy: torch.Tensor, params: List[torch.Tensor],
                               uid: int, flags: int, drop: float, seed: int,
                               need_dx: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """DSTDGCN backward -> dstd_model_train_bwd_ex."""
    m = _instance(uid)
    arena = native.GradArena(m._tree.get(m)[0], x.device)  # (see dstdgcb_train_backward)
    dx = _model_train_bwd_native(m, x, saved, dy, flags, drop, seed, m._native_grads(arena), need_dx)
    return (dx if dx is not None else x.new_empty(0)), arena.buf


@_op_dstdgcn_train_backward.register_fake
def _(x, saved, dy, params, uid, flags, drop, seed, need_dx):
    return (torch.empty_like(x) if need_dx else x.new_empty(0)), x.new_empty(native.arena_numel(params))


@torch.library.custom_op("dstd::dstdgc_train_forward", mutates_args=())
def _op_dstdgc_train_forward(x: torch.Tensor, A: torch.Tensor, alpha: torch.Tensor, weights: List[torch.Tensor],
                             uid: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """DSTDGC forward keeping the backward's state -> dstd_dstdgc_train_fwd."""
    mod = _instance(uid)
    mode = native.MODE_SPATIAL if mod.mode == "spatial" else native.MODE_TEMPORAL
    return _op_train_fwd_native(mod, mode, x, A, alpha)


@_op_dstdgc_train_forward.register_fake
def _(x, A, alpha, weights, uid):
    mod = _instance(uid)
    mode = native.MODE_SPATIAL if mod.mode == "spatial" else native.MODE_TEMPORAL
    B, cin, T, V = x.shape
    nbytes = native.lib().dstd_dstdgc_train_saved_bytes_r(mode, B, cin, mod.out_channels, T, V, mod.red_channels)
    return x.new_empty(B, mod.out_channels, T, V), x.new_empty(nbytes, dtype=torch.uint8)


@torch.library.custom_op("dstd::dstdgc_train_backward", mutates_args=())
def _op_dstdgc_train_backward(x: torch.Tensor, A: torch.Tensor, alpha: torch.Tensor, saved: torch.Tensor,
                              dy: torch.Tensor, weights: List[torch.Tensor], uid: int,
                              need_dx: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """DSTDGC backward -> dstd_dstdgc_train_bwd: (dx, dA, dalpha, weight-gradient arena)."""
    L = native.lib()
    mod = _instance(uid)
    mode = native.MODE_SPATIAL if mod.mode == "spatial" else native.MODE_TEMPORAL
    B, cin, T, V = x.shape
    dev = x.device
    cout = mod.out_channels
    arena = native.GradArena(list(mod.parameters()), dev)  # (see dstdgcb_train_backward)
    dx = torch.zeros_like(x) if need_dx else x.new_empty(0)
    dA = torch.zeros_like(A)
    dalpha = torch.zeros_like(alpha)
    red = mod.red_channels
    ws = native.workspace(dev, L.dstd_dstdgc_train_workspace_bytes_r(mode, B, cin, cout, T, V, red))
    code = L.dstd_dstdgc_train_bwd_r(mode, native.ptr(x, "x"), B, cin, cout, T, V, red, native.gc_weights(mod),
                                     native.ptr(alpha, "alpha_m"), saved.data_ptr(), saved.numel(),
                                     native.ptr(dy, "dy"), dx.data_ptr() if need_dx else None,
                                     native.gc_grads(mod, arena), native.ptr(dA, "dA"), native.ptr(dalpha, "dalpha"),
                                     ws.data_ptr(), ws.numel(), native.stream_handle(dev))
    native.check(code, "dstd_dstdgc_train_bwd_r")
    return dx, dA, dalpha, arena.buf


@_op_dstdgc_train_backward.register_fake
def _(x, A, alpha, saved, dy, weights, uid, need_dx):
    return ((torch.empty_like(x) if need_dx else x.new_empty(0)), torch.empty_like(A), torch.empty_like(alpha),
            x.new_empty(native.arena_numel(weights)))
