"""ctypes binding of the MI355X C ABI (include/dstd_gcn.h).

The shared library ``libdstd_gcn.so`` is built in-tree (``make -C dstd-gcn_amd``
or ``__graft_entry__.build()``).  There is no fallback: if the library is
missing or a tensor is not on a ROCm device, the call raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DSTD_LIB overrides the library (A/B experiments with variant builds)
LIB_PATH = os.environ.get("DSTD_LIB") or os.path.join(os.path.dirname(_HERE), "libdstd_gcn.so")

MODE_SPATIAL = 0
MODE_TEMPORAL = 1
MAX_LAYERS = 16

_fp = ctypes.POINTER(ctypes.c_float)


class GCWeights(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("wf", "bf", "wm1", "bm1", "wm2", "bm2", "wrm", "brm")]


class BN(ctypes.Structure):
    _fields_ = [("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("running_mean", ctypes.c_void_p),
                ("running_var", ctypes.c_void_p), ("eps", ctypes.c_float)]


class BlockParams(ctypes.Structure):
    _fields_ = [("cin", ctypes.c_int), ("cout", ctypes.c_int),
                ("A_s", ctypes.c_void_p), ("W_s", ctypes.c_void_p), ("R_s", ctypes.c_void_p),
                ("A_t", ctypes.c_void_p), ("R_t", ctypes.c_void_p),
                ("alpha_sm", ctypes.c_void_p), ("alpha_tm", ctypes.c_void_p),
                ("conv_s", GCWeights * 2), ("conv_t", GCWeights), ("bn", BN), ("prelu", ctypes.c_void_p),
                ("res_w", ctypes.c_void_p), ("res_b", ctypes.c_void_p), ("res_bn", BN)]


class ModelParams(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int), ("V", ctypes.c_int), ("num_layers", ctypes.c_int),
                ("num_feature", ctypes.c_int), ("in_channels", ctypes.c_int),
                ("st_in", BlockParams), ("bn_in", BN), ("prelu", ctypes.c_void_p),
                ("enc", BlockParams * MAX_LAYERS), ("enc_bn", BN * MAX_LAYERS),
                ("enc_prelu", ctypes.c_void_p * MAX_LAYERS), ("st_out", BlockParams)]


class Profile(ctypes.Structure):
    _fields_ = [("kind_mask", ctypes.c_uint), ("capacity", ctypes.c_int), ("count", ctypes.c_int),
                ("events", ctypes.POINTER(ctypes.c_void_p)), ("kinds", ctypes.POINTER(ctypes.c_int)),
                ("block", ctypes.POINTER(ctypes.c_int)), ("only_block", ctypes.c_int)]


class GCGrads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("wf", "bf", "wm1", "bm1", "wm2", "bm2", "wrm", "brm")]


class BNGrads(ctypes.Structure):
    _fields_ = [("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p)]


class BlockGrads(ctypes.Structure):
    _fields_ = [("W_s", ctypes.c_void_p), ("R_s", ctypes.c_void_p), ("R_t", ctypes.c_void_p),
                ("alpha_sm", ctypes.c_void_p), ("alpha_tm", ctypes.c_void_p),
                ("conv_s", GCGrads * 2), ("conv_t", GCGrads), ("bn", BNGrads), ("prelu", ctypes.c_void_p),
                ("res_w", ctypes.c_void_p), ("res_b", ctypes.c_void_p), ("res_bn", BNGrads)]


class ModelGrads(ctypes.Structure):
    _fields_ = [("st_in", BlockGrads), ("bn_in", BNGrads), ("prelu", ctypes.c_void_p),
                ("enc", BlockGrads * MAX_LAYERS), ("enc_bn", BNGrads * MAX_LAYERS),
                ("enc_prelu", ctypes.c_void_p * MAX_LAYERS), ("st_out", BlockGrads)]


# include/dstd_gcn_train.h dstd_bn_sync: cross-rank BatchNorm (dstd_dist.BnSync)
COLL_ALLGATHER, COLL_ALLREDUCE_SUM = 0, 1
COLLECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                 ctypes.c_void_p)


class BnSyncStruct(ctypes.Structure):
    _fields_ = [("world", ctypes.c_int), ("rank", ctypes.c_int), ("fn", COLLECTIVE_FN), ("ctx", ctypes.c_void_p),
                ("buf", ctypes.c_void_p), ("buf_floats", ctypes.c_longlong)]


TRAIN_RUNNING_STATS = 1  # include/dstd_gcn_train.h DSTD_TRAIN_RUNNING_STATS
TRAIN_PAIRED = 2  # DSTD_TRAIN_PAIRED: two BatchNorm batches of B/2 (a forward pair)
TRAIN_SEED_DEVICE = 4  # DSTD_TRAIN_SEED_DEVICE: the dropout seed is read from device memory
TRAIN_ONE_STREAM = 8  # DSTD_TRAIN_ONE_STREAM: no weight-gradient stream in the model backward
FWD_REUSE_CONSTANTS = 1  # include/dstd_gcn.h DSTD_FWD_REUSE_CONSTANTS
FWD_EXACT_FP32 = 2  # include/dstd_gcn.h DSTD_FWD_EXACT_FP32
FWD_SEPARATE_ADJ = 4  # include/dstd_gcn.h DSTD_FWD_SEPARATE_ADJ
FWD_FUSED_TEMPORAL = 8  # include/dstd_gcn.h DSTD_FWD_FUSED_TEMPORAL
FWD_SEPARATE_BLOCK = 16  # include/dstd_gcn.h DSTD_FWD_SEPARATE_BLOCK
KIND_FOLD, KIND_PREP, KIND_ADJ_S, KIND_SPATIAL, KIND_ADJ_T, KIND_TEMPORAL, KIND_BLOCK = range(7)
KIND_NAMES = ("fold", "prep", "adj_spatial", "spatial_gc", "adj_temporal", "temporal_gc", "block")

_lib = None


def source_hash():
    """sha256 (16 hex digits) of the sources the library is built from, in the
    order dstd-gcn_amd/Makefile hashes them (HASHED); None when the sources
    are not next to the package."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    rel = [os.path.relpath(p, pkg) for pat in ("csrc/*.hip", "csrc/*.h", "../include/*.h")
           for p in glob.glob(os.path.join(pkg, pat))]
    files = sorted(rel) + ["Makefile"]
    h = hashlib.sha256()
    for f in files:
        path = os.path.join(pkg, f)
        if not os.path.exists(path):
            return None
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def lib():
    """Load libdstd_gcn.so once; raise loudly if it is not built, or if it was
    built from other sources than the tree it is loaded from (its embedded
    dstd_source_hash() against source_hash())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"DSTD native library not built: {LIB_PATH} (run `make -C dstd-gcn_amd`)")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.dstd_source_hash.restype = ctypes.c_char_p
        built, tree = L.dstd_source_hash().decode(), source_hash()
        # DSTD_AB_FOREIGN_LIB=1: A/B tooling (scripts/ab_kernels.py) loading a
        # library built from an earlier revision on purpose
        if tree is not None and built != tree and os.environ.get("DSTD_AB_FOREIGN_LIB") != "1":
            raise RuntimeError(f"{LIB_PATH} was built from other sources (hash {built}, this tree {tree}): "
                               "rebuild with `make -C dstd-gcn_amd`")
        L.dstd_version.restype = ctypes.c_char_p
        L.dstd_error_string.restype = ctypes.c_char_p
        L.dstd_error_string.argtypes = [ci]
        L.dstd_dstdgc_workspace_bytes.restype = sz
        L.dstd_dstdgc_workspace_bytes.argtypes = [ci] * 6
        L.dstd_block_workspace_bytes.restype = sz
        L.dstd_block_workspace_bytes.argtypes = [ci] * 5
        L.dstd_model_workspace_bytes.restype = sz
        L.dstd_model_workspace_bytes.argtypes = [ci] * 5
        L.dstd_dstdgc_fwd.restype = ci
        L.dstd_dstdgc_fwd.argtypes = [ci, vp, ci, ci, ci, ci, ci, ctypes.POINTER(GCWeights), vp, vp, vp, vp, sz, vp]
        L.dstd_block_fwd.restype = ci
        L.dstd_block_fwd.argtypes = [ctypes.POINTER(BlockParams), vp, ci, ci, ci, vp, vp, sz, vp]
        L.dstd_block_fwd_ex.restype = ci
        L.dstd_block_fwd_ex.argtypes = [ctypes.POINTER(BlockParams), vp, ci, ci, ci, vp, vp, sz, vp, ctypes.c_uint]
        L.dstd_model_fwd.restype = ci
        L.dstd_model_fwd.argtypes = [ctypes.POINTER(ModelParams), vp, ci, vp, vp, sz, vp]
        L.dstd_model_fwd_ex.restype = ci
        L.dstd_model_fwd_ex.argtypes = [ctypes.POINTER(ModelParams), vp, ci, vp, vp, sz, vp, ctypes.c_uint,
                                        ctypes.POINTER(Profile)]
        L.dstd_model_fwd_profiled.restype = ci
        L.dstd_model_fwd_profiled.argtypes = [ctypes.POINTER(ModelParams), vp, ci, vp, vp, sz, vp,
                                              ctypes.POINTER(Profile)]
        L.dstd_events_create.restype = ci
        L.dstd_events_create.argtypes = [ci, ctypes.POINTER(ctypes.c_void_p)]
        L.dstd_events_destroy.restype = ci
        L.dstd_events_destroy.argtypes = [ci, ctypes.POINTER(ctypes.c_void_p)]
        L.dstd_event_elapsed_ms.restype = ci
        L.dstd_event_elapsed_ms.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_float)]
        # training path (include/dstd_gcn_train.h)
        u64, f32 = ctypes.c_ulonglong, ctypes.c_float
        for n, k in (("dstd_dstdgc_train_saved_bytes", 6), ("dstd_dstdgc_train_workspace_bytes", 6),
                     ("dstd_block_train_saved_bytes", 5), ("dstd_block_train_workspace_bytes", 5),
                     ("dstd_model_train_saved_bytes", 5), ("dstd_model_train_workspace_bytes", 5),
                     ("dstd_dstdgc_train_saved_bytes_r", 7), ("dstd_dstdgc_train_workspace_bytes_r", 7)):
            getattr(L, n).restype = sz
            getattr(L, n).argtypes = [ci] * k
        L.dstd_dstdgc_train_fwd.restype = ci
        L.dstd_dstdgc_train_fwd.argtypes = [ci, vp, ci, ci, ci, ci, ci, ctypes.POINTER(GCWeights), vp, vp, vp, vp, sz,
                                            vp]
        L.dstd_dstdgc_train_bwd.restype = ci
        L.dstd_dstdgc_train_bwd.argtypes = [ci, vp, ci, ci, ci, ci, ci, ctypes.POINTER(GCWeights), vp, vp, sz, vp, vp,
                                            ctypes.POINTER(GCGrads), vp, vp, vp, sz, vp]
        L.dstd_dstdgc_train_fwd_r.restype = ci
        L.dstd_dstdgc_train_fwd_r.argtypes = [ci, vp, ci, ci, ci, ci, ci, ci, ctypes.POINTER(GCWeights), vp, vp, vp,
                                              vp, sz, vp]
        L.dstd_dstdgc_train_bwd_r.restype = ci
        L.dstd_dstdgc_train_bwd_r.argtypes = [ci, vp, ci, ci, ci, ci, ci, ci, ctypes.POINTER(GCWeights), vp, vp, sz,
                                              vp, vp, ctypes.POINTER(GCGrads), vp, vp, vp, sz, vp]
        L.dstd_block_train_fwd.restype = ci
        L.dstd_block_train_fwd.argtypes = [ctypes.POINTER(BlockParams), vp, ci, ci, ci, f32, vp, vp, sz, vp]
        L.dstd_block_train_bwd.restype = ci
        L.dstd_block_train_bwd.argtypes = [ctypes.POINTER(BlockParams), vp, ci, ci, ci, vp, sz, vp, vp,
                                           ctypes.POINTER(BlockGrads), vp, sz, vp]
        L.dstd_model_train_fwd.restype = ci
        L.dstd_model_train_fwd.argtypes = [ctypes.POINTER(ModelParams), vp, ci, f32, f32, u64, vp, vp, sz, vp]
        L.dstd_model_train_bwd.restype = ci
        L.dstd_model_train_bwd.argtypes = [ctypes.POINTER(ModelParams), vp, ci, f32, u64, vp, sz, vp,
                                           ctypes.POINTER(ModelGrads), vp, sz, vp]
        uf = ctypes.c_uint
        L.dstd_block_train_fwd_ex.restype = ci
        L.dstd_block_train_fwd_ex.argtypes = L.dstd_block_train_fwd.argtypes + [uf]
        L.dstd_block_train_bwd_ex.restype = ci
        L.dstd_block_train_bwd_ex.argtypes = L.dstd_block_train_bwd.argtypes + [uf]
        L.dstd_model_train_fwd_ex.restype = ci
        L.dstd_model_train_fwd_ex.argtypes = L.dstd_model_train_fwd.argtypes + [uf]
        L.dstd_model_train_bwd_ex.restype = ci
        L.dstd_model_train_bwd_ex.argtypes = [ctypes.POINTER(ModelParams), vp, ci, f32, u64, vp, sz, vp,
                                              ctypes.POINTER(ModelGrads), vp, vp, sz, vp, uf]
        # (absent from a round-3 library loaded for an A/B: only SyncBN calls them)
        if hasattr(L, "dstd_bn_sync_buffer_floats"):
            L.dstd_bn_sync_buffer_floats.restype = sz
            L.dstd_bn_sync_buffer_floats.argtypes = [ci, ci, ci]
            L.dstd_model_train_fwd_sync.restype = ci
            L.dstd_model_train_fwd_sync.argtypes = L.dstd_model_train_fwd_ex.argtypes + [ctypes.POINTER(BnSyncStruct)]
            L.dstd_model_train_bwd_sync.restype = ci
            L.dstd_model_train_bwd_sync.argtypes = L.dstd_model_train_bwd_ex.argtypes + [ctypes.POINTER(BnSyncStruct)]
        L.dstd_loss_workspace_bytes.restype = sz
        L.dstd_loss_workspace_bytes.argtypes = []
        L.dstd_mpjpe_fwd.restype = ci
        L.dstd_mpjpe_fwd.argtypes = [vp, vp, sz, vp, vp, sz, vp]
        L.dstd_mpjpe_bwd.restype = ci
        L.dstd_mpjpe_bwd.argtypes = [vp, vp, sz, vp, f32, vp, vp]
        L.dstd_frame_mpjpe.restype = ci
        L.dstd_frame_mpjpe.argtypes = [vp, vp, ci, ci, ci, ci, vp, ci, vp, vp, ci, vp, vp]
        # non-refine ST_GCNN_layer branch (include/dstd_gcn_aux.h)
        L.dstd_ctg_workspace_bytes.restype = sz
        L.dstd_ctg_workspace_bytes.argtypes = [ci] * 4
        L.dstd_ctg_fwd.restype = ci
        L.dstd_ctg_fwd.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, vp, vp, sz, vp]
        L.dstd_ctg_bwd.restype = ci
        L.dstd_ctg_bwd.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
        L.dstd_conv2d_workspace_bytes.restype = sz
        L.dstd_conv2d_workspace_bytes.argtypes = [ci] * 11
        L.dstd_conv2d_fwd.restype = ci
        L.dstd_conv2d_fwd.argtypes = [vp, ci, ci, ci, ci, vp, vp] + [ci] * 7 + [vp, vp, sz, vp]
        L.dstd_conv2d_bwd.restype = ci
        L.dstd_conv2d_bwd.argtypes = [vp, ci, ci, ci, ci, vp] + [ci] * 7 + [vp, vp, vp, vp, vp, sz, vp]
        _lib = L
    return _lib


EXPORTS = ("dstd_version", "dstd_source_hash", "dstd_error_string", "dstd_dstdgc_workspace_bytes", "dstd_block_workspace_bytes",
           "dstd_model_workspace_bytes", "dstd_dstdgc_fwd", "dstd_block_fwd", "dstd_model_fwd",
           "dstd_model_fwd_profiled", "dstd_events_create", "dstd_events_destroy", "dstd_event_elapsed_ms",
           "dstd_block_fwd_ex", "dstd_model_fwd_ex")
TRAIN_EXPORTS = ("dstd_dstdgc_train_saved_bytes", "dstd_dstdgc_train_workspace_bytes", "dstd_dstdgc_train_fwd",
                 "dstd_dstdgc_train_bwd", "dstd_block_train_saved_bytes", "dstd_block_train_workspace_bytes",
                 "dstd_block_train_fwd", "dstd_block_train_bwd", "dstd_model_train_saved_bytes",
                 "dstd_model_train_workspace_bytes", "dstd_model_train_fwd", "dstd_model_train_bwd",
                 "dstd_loss_workspace_bytes", "dstd_mpjpe_fwd", "dstd_mpjpe_bwd", "dstd_frame_mpjpe",
                 "dstd_block_train_fwd_ex", "dstd_block_train_bwd_ex", "dstd_model_train_fwd_ex",
                 "dstd_model_train_bwd_ex", "dstd_dstdgc_train_saved_bytes_r",
                 "dstd_dstdgc_train_workspace_bytes_r", "dstd_dstdgc_train_fwd_r", "dstd_dstdgc_train_bwd_r",
                 "dstd_bn_sync_buffer_floats", "dstd_model_train_fwd_sync", "dstd_model_train_bwd_sync",
                 "dstd_debug_aggb_last")
AUX_EXPORTS = ("dstd_ctg_workspace_bytes", "dstd_ctg_fwd", "dstd_ctg_bwd", "dstd_conv2d_workspace_bytes",
               "dstd_conv2d_fwd", "dstd_conv2d_bwd")


ARITHMETICS = ("split", "fp32")


def arith_flags(mode):
    """Per-call flag of the graph-convolution arithmetic (include/dstd_gcn.h
    DSTD_FWD_EXACT_FP32): "split" (split-f16 MFMA where the shape has kernels,
    the default) or "fp32" (exact-fp32 MFMA everywhere)."""
    if mode not in ARITHMETICS:
        raise ValueError(f"gc arithmetic must be one of {ARITHMETICS}, got {mode!r}")
    return FWD_EXACT_FP32 if mode == "fp32" else 0


def check(code, what):
    if code != 0:
        msg = lib().dstd_error_string(code).decode()
        raise RuntimeError(f"{what} failed ({code}): {msg}")


# ---------------------------------------------------------------------------
# tensor helpers
# ---------------------------------------------------------------------------
def require_device(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: the DSTD path runs on the MI355X only (tensor is on {t.device}); "
                           "there is no CPU fallback")
    if t.dtype != torch.float32:
        raise ValueError(f"{name}: expected float32, got {t.dtype}")


def ptr(t, name="tensor"):
    require_device(t, name)
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    return t.data_ptr()


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_ws_cache = {}


def workspace(device, nbytes):
    """Caller-owned scratch (torch caching allocator), grown on demand and kept
    per (device, stream) so graph capture and steady state reuse one buffer."""
    return workspace_claim(device, nbytes, None)[0]


def workspace_claim(device, nbytes, tag):
    """workspace() for a caller that can reuse what its previous call left in
    the buffer: returns (buf, reused), reused = True iff the last claim of this
    buffer carried the same (non-None) tag and nothing else used it since."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    buf, last = _ws_cache.get(key, (None, None))
    reused = buf is not None and buf.numel() >= nbytes and tag is not None and last == tag
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
    _ws_cache[key] = (buf, tag)
    return buf, reused


def gc_weights(dstdgc):
    """GCWeights from a DSTDGC module (conv weights [O, I, 1, 1] are read as [O, I])."""
    w = GCWeights()
    for f, conv in (("f", dstdgc.conv_f), ("m1", dstdgc.conv_m1), ("m2", dstdgc.conv_m2), ("rm", dstdgc.conv_rm)):
        setattr(w, "w" + f, ptr(conv.weight, f"conv_{f}.weight"))
        setattr(w, "b" + f, ptr(conv.bias, f"conv_{f}.bias"))
    return w


def bn_struct(bnw):
    """BN from the reference BatchNorm wrapper (.bn = BatchNorm1d(C*V))."""
    b = bnw.bn
    return BN(ptr(b.weight, "bn.weight"), ptr(b.bias, "bn.bias"), ptr(b.running_mean, "bn.running_mean"),
              ptr(b.running_var, "bn.running_var"), float(b.eps))


def block_struct(blk):
    p = BlockParams()
    p.cin, p.cout = blk.in_channels, blk.out_channels
    p.A_s, p.W_s, p.R_s = ptr(blk.A_s, "A_s"), ptr(blk.W_s, "W_s"), ptr(blk.R_s, "R_s")
    p.A_t, p.R_t = ptr(blk.A_t, "A_t"), ptr(blk.R_t, "R_t")
    p.alpha_sm, p.alpha_tm = ptr(blk.alpha_sm, "alpha_sm"), ptr(blk.alpha_tm, "alpha_tm")
    p.conv_s[0] = gc_weights(blk.conv_s[0])
    p.conv_s[1] = gc_weights(blk.conv_s[1])
    p.conv_t = gc_weights(blk.conv_t[0])
    p.bn = bn_struct(blk.bn)
    p.prelu = ptr(blk.prelu.weight, "prelu.weight")
    if blk.in_channels != blk.out_channels:
        conv, bnw = blk.residual[0], blk.residual[1]
        p.res_w, p.res_b = ptr(conv.weight, "residual.0.weight"), ptr(conv.bias, "residual.0.bias")
        p.res_bn = bn_struct(bnw)
    return p


# ---------------------------------------------------------------------------
# gradient structs (training path)
# ---------------------------------------------------------------------------
class GradArena:
    """One zeroed fp32 buffer with a slice per parameter (the backward kernels
    accumulate into it); ``ptr(p)`` is p's slice, ``views()`` the gradients in
    the order given, None for parameters that do not require grad (A_s, A_t
    and anything frozen)."""

    def __init__(self, params, device, buf=None):
        self.params = list(params)
        self.offsets = {}
        n = 0
        for p in self.params:
            if id(p) not in self.offsets:
                self.offsets[id(p)] = n
                n += (p.numel() + 63) // 64 * 64
        if buf is not None:  # an arena a backward op returned (same params, same layout)
            if buf.numel() != max(n, 1):
                raise ValueError(f"gradient arena of {buf.numel()} floats for a layout of {max(n, 1)}")
            self.buf = buf
        else:
            self.buf = torch.zeros(max(n, 1), dtype=torch.float32, device=device)

    def ptr(self, p):
        return self.buf.data_ptr() + 4 * self.offsets[id(p)]

    def views(self):
        out = []
        for p in self.params:
            off = self.offsets[id(p)]
            out.append(self.buf[off:off + p.numel()].view(p.shape) if p.requires_grad else None)
        return out


def arena_numel(params):
    """Floats of a GradArena over ``params`` (64-float aligned slices, shared
    tensors once)."""
    seen, n = set(), 0
    for p in params:
        if id(p) not in seen:
            seen.add(id(p))
            n += (p.numel() + 63) // 64 * 64
    return max(n, 1)


def grad_sink(owner, params, device):
    """Where a native backward writes the parameters' gradients.

    Returns (arena, direct).  direct=True: the parameters' ``.grad`` ARE
    slices of ``owner``'s persistent arena and the backward kernels, which
    always accumulate (+=), add into them in place -- the caller returns None
    to autograd for the parameters.  That is torch's accumulate semantics
    without a per-parameter clone / add kernel per backward (a training step
    with the inverse pass runs two backwards into the same gradients:
    engine/prediction.py:267-287).  It holds when every trainable parameter's
    ``.grad`` is None (the arena is zeroed and the views installed) or is
    still the view installed earlier.  Otherwise (gradients set by someone
    else) a fresh zeroed arena is returned with direct=False and the caller
    hands its views to autograd as before."""
    params = params if isinstance(params, list) else list(params)
    dev = torch.device(device)
    arena = getattr(owner, "_dstd_grad_arena", None)
    if (arena is None or len(arena.params) != len(params) or arena.buf.device != dev
            or any(a is not b for a, b in zip(arena.params, params))):
        arena = GradArena(params, device)
        # (parameter, its slice) for every trainable parameter, built once
        arena.pairs = [(q, v) for q, v in zip(arena.params, arena.views()) if v is not None]
        owner._dstd_grad_arena = arena
    pairs = arena.pairs
    grads = [q.grad for q, _ in pairs]
    if all(g is None for g in grads):
        arena.buf.zero_()
        for q, v in pairs:
            q.grad = v
        return arena, True
    if all(g is v for g, (_, v) in zip(grads, pairs)):
        return arena, True
    return GradArena(params, device), False


def gc_grads(dstdgc, arena):
    g = GCGrads()
    for f, conv in (("f", dstdgc.conv_f), ("m1", dstdgc.conv_m1), ("m2", dstdgc.conv_m2), ("rm", dstdgc.conv_rm)):
        setattr(g, "w" + f, arena.ptr(conv.weight))
        setattr(g, "b" + f, arena.ptr(conv.bias))
    return g


def bn_grads(bnw, arena):
    return BNGrads(arena.ptr(bnw.bn.weight), arena.ptr(bnw.bn.bias))


def block_grads(blk, arena):
    g = BlockGrads()
    g.W_s, g.R_s, g.R_t = arena.ptr(blk.W_s), arena.ptr(blk.R_s), arena.ptr(blk.R_t)
    g.alpha_sm, g.alpha_tm = arena.ptr(blk.alpha_sm), arena.ptr(blk.alpha_tm)
    g.conv_s[0] = gc_grads(blk.conv_s[0], arena)
    g.conv_s[1] = gc_grads(blk.conv_s[1], arena)
    g.conv_t = gc_grads(blk.conv_t[0], arena)
    g.bn = bn_grads(blk.bn, arena)
    g.prelu = arena.ptr(blk.prelu.weight)
    if blk.in_channels != blk.out_channels:
        g.res_w, g.res_b = arena.ptr(blk.residual[0].weight), arena.ptr(blk.residual[0].bias)
        g.res_bn = bn_grads(blk.residual[1], arena)
    return g
