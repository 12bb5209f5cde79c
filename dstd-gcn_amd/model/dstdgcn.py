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

There is no CPU / eager fallback: a tensor off the GPU, a missing library or a
train-mode call raises.  Train mode (batch-statistics BatchNorm and the
backward pass) is not built yet and raises
NotImplementedError; outputs carry a grad_fn whose backward raises, so a
silent zero gradient is impossible.
"""
import math

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
    """Marks native outputs: forward is identity, backward refuses loudly."""

    @staticmethod
    def forward(ctx, y, *deps):
        return y

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError("DSTD native backward kernels are not built yet (SURVEY §8(f) row 1); "
                                  "gradients through the MI355X forward are unavailable")


def _mark(y, *deps):
    if torch.is_grad_enabled():
        req = [d for d in deps if isinstance(d, torch.Tensor) and d.requires_grad]
        if req:
            return _ForwardOnly.apply(y, *req)
    return y


def _no_train(module):
    if module.training:
        raise NotImplementedError(f"{type(module).__name__}: train-mode forward (batch-statistics BatchNorm + "
                                  "backward) is not built yet (SURVEY §8(f) row 1); call .eval()")


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


class DSTDGC(nn.Module):
    """Dynamic graph convolution (reference :53-94); ``mode`` spatial or temporal."""

    def __init__(self, in_channels, out_channels, ref_channels, kpt_channels, red_channels=2, mode="spatial"):
        super().__init__()
        if mode not in ("spatial", "temporal"):
            raise AssertionError(f"mode must be spatial or temporal, got {mode}")
        if red_channels != 2:
            raise NotImplementedError("the MI355X kernels are built for red_channels == 2 (every shipped config)")
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
        A = A.reshape(A.shape[-2], A.shape[-1]).contiguous()
        if not torch.is_tensor(alpha_m):
            alpha_m = torch.full((1,), float(alpha_m), dtype=torch.float32, device=dev)
        alpha = alpha_m.reshape(1).contiguous()
        mode = native.MODE_SPATIAL if self.mode == "spatial" else native.MODE_TEMPORAL
        y = torch.empty(B, self.out_channels, T, V, dtype=torch.float32, device=dev)
        nbytes = L.dstd_dstdgc_workspace_bytes(mode, B, cin, self.out_channels, T, V)
        ws = native.workspace(dev, nbytes)
        w = native.gc_weights(self)
        code = L.dstd_dstdgc_fwd(mode, native.ptr(x, "x"), B, cin, self.out_channels, T, V, w,
                                 native.ptr(A, "A"), native.ptr(alpha, "alpha_m"), native.ptr(y, "y"),
                                 ws.data_ptr(), ws.numel(), native.stream_handle(dev))
        native.check(code, "dstd_dstdgc_fwd")
        return _mark(y, x, A, alpha, *self.parameters())


class DSTDGCB(nn.Module):
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

    def init_parameter(self):
        stdt = 1.0 / math.sqrt(self.R_t.size(1))
        self.R_t.data.uniform_(-stdt, stdt)
        stdt = 1.0 / math.sqrt(self.R_s.size(1))
        self.R_s.data.uniform_(-stdt, stdt)

    def forward(self, x):
        _no_train(self)
        L = native.lib()
        B, cin, T, V = x.shape
        x = x.contiguous()
        native.require_device(x, "x")
        dev = x.device
        y = torch.empty(B, self.out_channels, T, V, dtype=torch.float32, device=dev)
        nbytes = L.dstd_block_workspace_bytes(B, cin, self.out_channels, T, V)
        ws = native.workspace(dev, nbytes)
        p = native.block_struct(self)
        code = L.dstd_block_fwd(p, native.ptr(x, "x"), B, T, V, native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                                native.stream_handle(dev))
        native.check(code, "dstd_block_fwd")
        return _mark(y, x, *self.parameters())


class ST_GCNN_layer(nn.Module):
    """Wrapper of one DSTDGCB plus an optional residual (reference :191-249).
    Only ``refine=True`` exists in the shipped configs; the STS-GCN style
    ``refine=False`` branch (ConvTemporalGraphical) is not built."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, time_dim, joints_dim, bias=True,
                 refine=False, residual=True, layout="h36m"):
        super().__init__()
        self.kernel_size = kernel_size
        self.refine = refine
        assert self.kernel_size[0] % 2 == 1
        assert self.kernel_size[1] % 2 == 1
        if not refine:
            raise NotImplementedError("ST_GCNN_layer(refine=False) (ConvTemporalGraphical) is unreachable in the "
                                      "shipped configs and not built (SURVEY §8(f) row 4)")
        self.stgcn = nn.ModuleList([nn.Sequential(DSTDGCB(in_channels, out_channels, time_dim, joints_dim, layout))])
        if not residual:
            self.residual = None
        elif stride != 1 or in_channels != out_channels:
            self.residual = nn.Conv2d(in_channels, out_channels, kernel_size=1, stride=1)
        else:
            self.residual = nn.Identity()
        self.apply(weights_init)

    def forward(self, x):
        y = None
        for stb in self.stgcn:
            z = stb(x)
            y = z if y is None else y + z
        if self.residual is not None:
            y = y + self.residual(x)
        return y


class DSTDGCN(nn.Module):
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

    # -- native parameter block ---------------------------------------------
    def _native_params(self):
        tensors = list(self.parameters()) + list(self.buffers())
        ptrs = [t.data_ptr() for t in tensors]
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
        self._native = (ptrs, p)
        return p

    def forward(self, x):
        n, t, v, c = x.shape
        assert t == self.input_time_frame + self.output_time_frame
        _no_train(self)
        if c != self.input_channels // 2 or v != self.joints_to_consider:
            raise ValueError(f"DSTDGCN: expected [N, {t}, {self.joints_to_consider}, {self.input_channels // 2}], "
                             f"got {list(x.shape)}")
        L = native.lib()
        x = x.contiguous()
        native.require_device(x, "x")
        dev = x.device
        p = self._native_params()
        y = torch.empty_like(x)
        nbytes = L.dstd_model_workspace_bytes(n, t, v, self.num_feature, self.num_layers)
        ws = native.workspace(dev, nbytes)
        code = L.dstd_model_fwd(p, native.ptr(x, "x"), n, native.ptr(y, "y"), ws.data_ptr(), ws.numel(),
                                native.stream_handle(dev))
        native.check(code, "dstd_model_fwd")
        return _mark(y, x, *self.parameters())
