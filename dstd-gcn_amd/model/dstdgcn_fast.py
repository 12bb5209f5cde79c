"""The channels-last DSTD-GCN variant -- drop-in for the reference's
``model/dstdgcn_fast.py`` (selected there by switching the import in
``model/__init__.py:7-8``; here ``from model.dstdgcn_fast import DSTDGCN``).

Same class names, constructor signatures, sub-module names and parameter
names / shapes / registration order as the reference file, so its
``state_dict`` loads unchanged.  The variant differs from ``model/dstdgcn.py``
in its schema and layout, not in the network:

  * activations are NTVC ``[N, T, V, C]`` end to end (:115, :134);
  * ``conv_f`` and the block residual are ``nn.Linear`` (:95, :185);
  * the spatial adjacency is the trainable ``A_s`` itself -- no ``W_s`` /
    ``R_s`` (:175, :256);
  * BatchNorm channels are ordered (v, c) (:53);
  * the graph product contracts the adjacency's SECOND index,
    ``matmul(xm, xf)`` (:125, :145), where dstdgcn.py contracts its first.

Because tanh is odd, the last point is the dstdgcn.py operator on remapped
weights:  M_fast[v][w] = a(W tanh(m1[v] - m2[w]) + b) + A[v][w] equals
M[w][v] for m1' = m2, m2' = m1, W' = -W, b' = b, A' = A^T.  So every module
here runs on the MI355X kernels of dstdgcn.py through a private *shadow*
module of the dstdgcn.py schema whose tensors are derived from this module's
(``_links``):

  conv_m1 <-> conv_m2 swapped, conv_rm.weight negated, conv_f / residual
  Linear weights as 1x1 convs, A_s^T as R_s (W_s = 0), A_t^T / R_t^T,
  BN vectors permuted (v, c) -> (c, v).

Eval forwards re-derive the shadow only when a tensor changed (torch version
counters, storage, the cache generation -- ``invalidate_native_cache``), then
run the shadow's single C call (``dstd_model_fwd_ex`` for the model).  The
training path (and an eval forward under autograd) runs the shadow's native autograd Functions with the derived
tensors as their inputs, so autograd carries the native gradients back
through the (linear) derivation onto this module's parameters, and the
shadow's updated BN running statistics are written back after each
train-mode forward.
"""
import math

import torch
import torch.nn as nn

import dstd_native as native

from . import dstdgcn as base
from .dstdgcn import ConvTemporalGraphical, Conv2d, bn_init, conv_init, weights_init  # noqa: F401  (reference names)
from .layers.graph import Graph
from .layers.time import Time


class BatchNorm(nn.Module):
    """BN1d over V*C channels of an NTVC tensor, channel index v*C + c
    (reference dstdgcn_fast.py:41-56).  Glue only: inside a DSTDGCB / DSTDGCN
    forward every BatchNorm is folded into the native kernels' epilogues."""

    def __init__(self, feature_channels, joint_dim, time_dim):
        super().__init__()
        self.c = feature_channels
        self.v = joint_dim
        self.t = time_dim
        self.bn = nn.BatchNorm1d(feature_channels * joint_dim)

    def forward(self, x):
        n, t, v, c = x.shape
        assert (c, t, v) == (self.c, self.t, self.v)
        y = self.bn(x.permute(0, 2, 3, 1).reshape(n, c * v, t))
        return y.reshape(n, v, c, t).permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------
# shadow modules: the dstdgcn.py schema, derived from the fast tensors
# ---------------------------------------------------------------------------
def _bn_to_base(f, c, v):
    return f.reshape(v, c).t().reshape(-1)  # [v*C + c] -> [c*V + v]


def _bn_from_base(s, c, v):
    return s.reshape(c, v).t().reshape(-1)


def _links(fast, shadow):
    """For every parameter and buffer of ``shadow`` (in its parameters() /
    buffers() order): (kind, fast tensors, derive), derive(*fast tensors) ->
    the shadow tensor.  The derivations are linear, so autograd through them
    maps the shadow's gradients back onto the fast parameters."""
    fmods = dict(fast.named_modules())
    out = []

    def owner(name):
        return name.rsplit(".", 1) if "." in name else ("", name)

    def link(name):
        mpath, leaf = owner(name)
        smod = shadow.get_submodule(mpath)
        if isinstance(smod, nn.BatchNorm1d):  # BN wrapper ".bn": permute (v, c) -> (c, v)
            wrap = fmods[mpath.rsplit(".", 1)[0] if "." in mpath else ""]
            src = getattr(fmods[mpath], leaf)
            if leaf == "num_batches_tracked":
                return [src], lambda f: f
            return [src], lambda f, c=wrap.c, v=wrap.v: _bn_to_base(f, c, v)
        if isinstance(smod, (base.DSTDGCB,)):
            if leaf in ("A_s", "R_s"):  # the fast A_s is the whole spatial adjacency
                return [fmods[mpath].A_s], lambda f: f.transpose(-1, -2)
            if leaf == "W_s":
                return [], lambda z=torch.zeros_like(smod.W_s): z
            if leaf in ("A_t", "R_t"):
                return [getattr(fmods[mpath], leaf)], lambda f: f.transpose(-1, -2)
            return [getattr(fmods[mpath], leaf)], lambda f: f  # alpha_sm, alpha_tm
        if isinstance(smod, nn.Conv2d):
            cpath, conv = owner(mpath)
            if conv in ("conv_m1", "conv_m2") and isinstance(shadow.get_submodule(cpath), base.DSTDGC):
                other = "conv_m2" if conv == "conv_m1" else "conv_m1"
                return [getattr(fmods[f"{cpath}.{other}" if cpath else other], leaf)], lambda f: f
            fsrc = getattr(fmods[mpath], leaf)
            if conv == "conv_rm" and leaf == "weight":
                return [fsrc], lambda f: -f
            if isinstance(fmods[mpath], nn.Linear) and leaf == "weight":  # conv_f / residual.0
                return [fsrc], lambda f: f.reshape(f.shape[0], f.shape[1], 1, 1)
            return [fsrc], lambda f: f
        return [getattr(fmods[mpath], leaf)], lambda f: f  # PReLU slopes, plain-layer tensors

    for name, _ in shadow.named_parameters():
        out.append(("param",) + tuple(link(name)))
    for name, _ in shadow.named_buffers():
        out.append(("buffer",) + tuple(link(name)))
    return out


def _mapped(fn):
    """A native autograd Function of dstdgcn.py run on a shadow module whose
    parameters are set from derived tensors: same argument positions as
    ``fn`` with the derived tensors in place of the shadow's parameters, so
    its backward's gradients land on them."""

    class _Mapped(torch.autograd.Function):
        @staticmethod
        def forward(ctx, mod, *rest):
            params = mod._dstd_shadow_params
            k = len(rest) - len(params)
            with torch.no_grad():
                for p, t in zip(params, rest[k:]):
                    if p.data_ptr() != t.data_ptr():
                        p.copy_(t)
            return fn.forward(ctx, mod, *rest[:k], *params)

        @staticmethod
        def backward(ctx, *grads):
            return fn.backward(ctx, *grads)

    _Mapped.__name__ = f"_Mapped{fn.__name__}"
    return _Mapped


_OpTrainM, _BlockTrainM, _ModelTrainM = _mapped(base._OpTrain), _mapped(base._BlockTrain), _mapped(base._ModelTrain)


class _Shadowed(nn.Module):
    """Owns the private dstdgcn.py-schema module (not a registered child: it
    is not in state_dict() / parameters()) and keeps it derived from self."""

    def _init_shadow(self, *args, **kwargs):
        self.__dict__["_shadow"] = None
        self.__dict__["_shadow_args"] = (args, kwargs)
        self.__dict__["_shadow_tag"] = None
        self._dstd_gen = 0

    def __getstate__(self):
        state = super().__getstate__() if hasattr(super(), "__getstate__") else self.__dict__.copy()
        state = dict(state)
        state["_shadow"], state["_shadow_tag"] = None, None
        return state

    def _make_shadow(self):
        raise NotImplementedError

    def _shadow_for(self, device):
        sh = self.__dict__.get("_shadow")
        if sh is None or sh._dstd_device != device:
            with torch.random.fork_rng(devices=[]):  # the shadow's own init must not move the caller's RNG
                sh = self._make_shadow().to(device)
            sh._dstd_device = device
            sh._dstd_links = _links(self, sh)
            sh._dstd_shadow_params = list(sh.parameters())
            self.__dict__["_shadow"] = sh
            self.__dict__["_shadow_tag"] = None
        sh.train(self.training)
        if hasattr(sh, "set_gc_arithmetic"):
            sh.set_gc_arithmetic(self.gc_arithmetic)
        elif hasattr(sh, "gc_arithmetic"):
            sh.gc_arithmetic = self.gc_arithmetic
        return sh

    def _tensors_tag(self):
        ts = list(self.parameters()) + list(self.buffers())
        try:
            return (self._dstd_gen, tuple(t.data_ptr() for t in ts), tuple(t._version for t in ts))
        except RuntimeError:  # inference tensors carry no version counter: always re-derive
            return None

    def _sync(self, sh, params=True):
        """Re-derive the shadow's tensors (params and buffers, or buffers only)
        unless nothing changed since the last full derivation."""
        tag = self._tensors_tag()
        if params and tag is not None and tag == self.__dict__.get("_shadow_tag"):
            return
        stensors = list(sh.parameters()) + list(sh.buffers())
        with torch.no_grad():
            for st, (kind, srcs, derive) in zip(stensors, sh._dstd_links):
                if kind == "param" and not params:
                    continue
                st.copy_(derive(*srcs))
        if params:
            self.__dict__["_shadow_tag"] = self._tensors_tag()

    def _derived_params(self, sh):
        """The shadow's parameters derived from self with autograd (training)."""
        return [derive(*srcs) for kind, srcs, derive in sh._dstd_links if kind == "param"]

    def _write_back_running_stats(self, sh):
        """Train-mode forwards update the shadow's BN statistics: copy them
        (permuted back to (v, c)) into this module's buffers."""
        fmods = dict(self.named_modules())
        with torch.no_grad():
            for name, sb in sh.named_buffers():
                mpath, leaf = name.rsplit(".", 1)
                fb = getattr(fmods[mpath], leaf)
                if leaf == "num_batches_tracked":
                    fb.copy_(sb)
                else:
                    wrap = fmods[mpath.rsplit(".", 1)[0] if "." in mpath else ""]
                    fb.copy_(_bn_from_base(sb, wrap.c, wrap.v))
        self.__dict__["_shadow_tag"] = self._tensors_tag()  # the shadow already holds these


class DSTDGC(_Shadowed):
    """Dynamic graph convolution, channels-last (reference dstdgcn_fast.py:59-155).
    x [N, T, V, Cin] -> [N, T, V, Cout]."""

    def __init__(self, in_channels, out_channels, ref_channels, kpt_channels, red_channels=2, mode="spatial"):
        super().__init__()
        assert mode in {"spatial", "temporal"}
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
        self.conv_f = nn.Linear(in_channels, out_channels)
        self.init_parameter()
        self._init_shadow()

    def init_parameter(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                conv_init(m)

    def _make_shadow(self):
        return base.DSTDGC(self.in_channels, self.out_channels, self.ref_channels, self.kpt_channels,
                           self.red_channels, self.mode)

    def forward(self, x, A=None, alpha_m=1):
        n, t, v, c = x.shape
        if c != self.in_channels:
            raise ValueError(f"DSTDGC: expected {self.in_channels} input channels, got {c}")
        native.require_device(x, "x")
        dev = x.device
        sh = self._shadow_for(dev)
        xs = x.permute(0, 3, 1, 2).contiguous()  # NCTV for the dstdgcn.py operator
        if n == 0:
            return x.new_empty(0, t, v, self.out_channels)
        At = A.reshape(A.shape[-2], A.shape[-1]).transpose(0, 1).contiguous()  # A' = A^T
        if not torch.is_tensor(alpha_m):
            alpha_m = torch.full((1,), float(alpha_m), dtype=torch.float32, device=dev)
        alpha = alpha_m.reshape(1).contiguous()
        mode = native.MODE_SPATIAL if self.mode == "spatial" else native.MODE_TEMPORAL
        params = list(self.parameters())
        if base._needs_grad(x, A, alpha, *params):
            y = _OpTrainM.apply(sh, mode, xs, At, alpha, *self._derived_params(sh))
        else:
            self._sync(sh)
            y = torch.ops.dstd.dstdgc_forward(xs, At, alpha, list(sh.parameters()), sh._dstd_uid)
        return y.permute(0, 2, 3, 1).contiguous()


class DSTDGCB(_Shadowed):
    """DSTD-GC block, channels-last (reference dstdgcn_fast.py:158-275).
    x [N, T, V, Cin] -> [N, T, V, Cout]."""

    def __init__(self, in_channels, out_channels, time_dim, joint_dim, layout="h36m"):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self._geom = (time_dim, joint_dim, layout)
        A_s = Graph(layout).get_all_adjacency()
        A_t = Time(time_dim).get_all_adjacency()
        # registration order follows the reference (:175-178)
        self.A_s = nn.Parameter(torch.tensor(A_s, dtype=torch.float32))
        self.A_t = nn.Parameter(torch.tensor(A_t, dtype=torch.float32), False)
        self.R_t = nn.Parameter(torch.zeros_like(self.A_t))
        self.conv_s = nn.ModuleList()
        self.conv_t = nn.ModuleList()
        if in_channels != out_channels:
            self.residual = nn.Sequential(nn.Linear(in_channels, out_channels),
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
        self.do = nn.Dropout(0.1)  # constructed but never applied (reference :227)
        self.gc_arithmetic = "split"  # as dstdgcn.DSTDGCB.gc_arithmetic
        self._init_shadow()

    def init_parameter(self):
        stdt = 1.0 / math.sqrt(self.R_t.size(1))
        self.R_t.data.uniform_(-stdt, stdt)

    def _make_shadow(self):
        T, V, layout = self._geom
        return base.DSTDGCB(self.in_channels, self.out_channels, T, V, layout)

    def forward(self, x):
        n, t, v, c = x.shape
        native.require_device(x, "x")
        sh = self._shadow_for(x.device)
        xs = x.permute(0, 3, 1, 2).contiguous()
        if self.training or base._needs_grad(x, *self.parameters()):
            # train mode, or eval under autograd (running-statistics BN)
            self._sync(sh, params=False)
            y = _BlockTrainM.apply(sh, xs, *self._derived_params(sh))
            if self.training:
                self._write_back_running_stats(sh)
        else:
            self._sync(sh)
            y = sh(xs)
        return y.permute(0, 2, 3, 1).contiguous()


class ST_GCNN_layer(nn.Module):
    """One fast DSTDGCB plus an optional residual (reference dstdgcn_fast.py:338-450).
    ``refine=False`` builds ConvTemporalGraphical + Conv2d as the reference
    does (dead code there too: those layers index dims as NCTV)."""

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
        if self.residual is not None:
            res = self.residual(x)
        if self.refine:
            y = None
            for stb in self.stgcn:
                z = stb(x)
                y = z if y is None else y + z
        else:
            y = self.stgcn(x)
        if self.residual is not None:
            y = y + res
        return y


class DSTDGCN(_Shadowed):
    """The whole channels-last network (reference dstdgcn_fast.py:453-614):
    x [N, T, V, 3] -> [N, T, V, 3], one native call per eval forward."""

    def __init__(self, input_channels, input_time_frame, output_time_frame, st_gcnn_dropout, joints_to_consider,
                 num_feature=64, num_layers=7, layout="h36m"):
        super().__init__()
        self.input_time_frame = input_time_frame
        self.output_time_frame = output_time_frame
        self.joints_to_consider = joints_to_consider
        self._ctor = (input_channels, input_time_frame, output_time_frame, st_gcnn_dropout, joints_to_consider,
                      num_feature, num_layers, layout)
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
        self.gc_arithmetic = "split"
        self._init_shadow()
        self.register_load_state_dict_post_hook(lambda mod, incompatible: base.invalidate_native_cache(mod))

    def set_gc_arithmetic(self, mode):
        """"split" (default) or "fp32" (include/dstd_gcn.h DSTD_FWD_EXACT_FP32)."""
        native.arith_flags(mode)
        for m in self.modules():
            if isinstance(m, (DSTDGCN, DSTDGCB)):
                m.gc_arithmetic = mode
        return self

    def _make_shadow(self):
        return base.DSTDGCN(*self._ctor)

    def forward(self, x):
        n, t, v, c = x.shape
        assert t == self.input_time_frame + self.output_time_frame
        native.require_device(x, "x")
        sh = self._shadow_for(x.device)
        sh.do_in.p = self.do_in.p
        if self.training or base._needs_grad(x, *self.parameters()):
            self._sync(sh, params=False)
            y = _ModelTrainM.apply(sh, False, x.contiguous(), *self._derived_params(sh))
            if self.training:
                self._write_back_running_stats(sh)
            return y
        self._sync(sh)
        return sh(x)

    def forward_pair(self, x1, x2):
        """``(self(x1), self(x2))`` as one paired native train step
        (dstdgcn.DSTDGCN.forward_pair: per-half BatchNorm statistics, running
        statistics updated in call order); the two calls outside train mode."""
        if not self.training or x1.shape != x2.shape or x1.shape[0] == 0 or x1.device != x2.device:
            return self(x1), self(x2)
        n, t, v, c = x1.shape
        assert t == self.input_time_frame + self.output_time_frame
        native.require_device(x1, "x")
        sh = self._shadow_for(x1.device)
        sh.do_in.p = self.do_in.p
        self._sync(sh, params=False)
        y = _ModelTrainM.apply(sh, True, torch.cat([x1, x2]).contiguous(), *self._derived_params(sh))
        self._write_back_running_stats(sh)
        return y[:n], y[n:]
