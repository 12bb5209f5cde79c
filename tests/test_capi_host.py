"""Host-side checks of the C ABI and the drop-in modules (no GPU needed)."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, group, load_npz
import dstd_native as native
from model import DSTDGC, DSTDGCB, DSTDGCN, get_model

H36M = dict(input_channels=6, input_time_frame=10, output_time_frame=25, st_gcnn_dropout=0.1,
            joints_to_consider=22, num_feature=64, num_layers=5, layout="h36m")


def header_symbols(name="dstd_gcn.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(dstd_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    L = native.lib()
    syms = header_symbols()
    assert len(syms) == 15, syms
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(native.EXPORTS)


def test_arithmetic_is_a_per_call_flag():
    """No process-wide arithmetic state: the choice travels with each call
    (DSTD_FWD_EXACT_FP32); unknown flag bits are rejected before any GPU work."""
    L = native.lib()
    assert not hasattr(L, "dstd_set_gc_precision")
    assert native.arith_flags("split") == 0 and native.arith_flags("fp32") == native.FWD_EXACT_FP32
    with pytest.raises(ValueError):
        native.arith_flags("bf16")
    assert L.dstd_block_fwd_ex(None, None, 4, 35, 22, None, None, 0, None, 4) == -1  # DSTD_EINVAL
    assert L.dstd_model_fwd_ex(None, None, 4, None, None, 0, None, 8, None) == -1
    m = get_model("dstdgcn", dstdgcn=H36M)
    assert m.gc_arithmetic == "split"
    m.set_gc_arithmetic("fp32")
    assert all(b.gc_arithmetic == "fp32" for b in m.modules() if isinstance(b, DSTDGCB))


def test_library_exports_every_training_header_symbol():
    L = native.lib()
    syms = header_symbols("dstd_gcn_train.h")
    assert len(syms) == 28, syms
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(native.TRAIN_EXPORTS)


def test_syncbn_buffer_and_error_without_gpu():
    """dstd_bn_sync (SyncBN): the buffer a caller allocates holds the forward's
    all-gather (world x 2 groups x C*V x (mean, M2, count)) and the backward's
    all-reduce; a failed collective has an error string of its own."""
    L = native.lib()
    assert L.dstd_bn_sync_buffer_floats(8, 64, 22) == 8 * 2 * 64 * 22 * 3
    assert L.dstd_bn_sync_buffer_floats(1, 64, 22) == 2 * 64 * 22 * 3
    assert L.dstd_bn_sync_buffer_floats(2, 64, 25) > L.dstd_bn_sync_buffer_floats(1, 64, 25)
    s = native.BnSyncStruct(2, 1, native.COLLECTIVE_FN(lambda *a: 0), None, 16, 1 << 20)
    assert (s.world, s.rank, s.buf_floats) == (2, 1, 1 << 20)
    assert "SyncBN" in L.dstd_error_string(-5).decode()


def test_train_sizes_and_argument_checks_without_gpu():
    L = native.lib()
    # saved activations grow linearly with the batch
    a = L.dstd_model_train_saved_bytes(8, 40, 23, 64, 5)
    b = L.dstd_model_train_saved_bytes(16, 40, 23, 64, 5)
    assert 0 < a < b and abs((b - a) - (a - L.dstd_model_train_saved_bytes(0, 40, 23, 64, 5))) < 1 << 20
    assert L.dstd_model_train_workspace_bytes(8, 40, 23, 64, 5) > 0
    assert L.dstd_block_train_saved_bytes(4, 6, 64, 35, 22) > L.dstd_block_train_saved_bytes(4, 64, 64, 35, 22) // 2
    assert L.dstd_dstdgc_train_saved_bytes(1, 4, 64, 64, 35, 22) > 0
    # red_channels: the red = 2 entry points are the _r ones at 2; more P / Q
    # channels, more saved state (the tanh planes grow with red)
    assert L.dstd_dstdgc_train_saved_bytes_r(1, 4, 64, 64, 35, 22, 2) == L.dstd_dstdgc_train_saved_bytes(
        1, 4, 64, 64, 35, 22)
    assert L.dstd_dstdgc_train_workspace_bytes_r(0, 4, 64, 64, 35, 22, 2) == L.dstd_dstdgc_train_workspace_bytes(
        0, 4, 64, 64, 35, 22)
    assert (L.dstd_dstdgc_train_saved_bytes_r(0, 4, 64, 64, 35, 22, 1) < L.dstd_dstdgc_train_saved_bytes_r(
        0, 4, 64, 64, 35, 22, 2) < L.dstd_dstdgc_train_saved_bytes_r(0, 4, 64, 64, 35, 22, 5))
    assert L.dstd_loss_workspace_bytes() > 0
    # null pointers / bad shapes are rejected before any device work
    w = native.GCWeights()
    g = native.GCGrads()
    assert L.dstd_dstdgc_train_fwd(0, None, 4, 64, 64, 35, 22, w, None, None, None, None, 0, None) == -1
    assert L.dstd_dstdgc_train_bwd(0, None, 4, 64, 64, 35, 22, w, None, None, 0, None, None, g, None, None, None, 0,
                                   None) == -1
    assert L.dstd_dstdgc_train_fwd_r(0, None, 4, 64, 64, 35, 22, 3, w, None, None, None, None, 0, None) == -1
    assert L.dstd_dstdgc_train_bwd_r(0, None, 4, 64, 64, 35, 22, 3, w, None, None, 0, None, None, g, None, None,
                                     None, 0, None) == -1
    assert L.dstd_block_train_fwd(None, None, 4, 35, 22, 0.1, None, None, 0, None) == -1
    assert L.dstd_model_train_fwd(None, None, 4, 0.1, 0.0, 0, None, None, 0, None) == -1
    assert L.dstd_model_train_bwd(None, None, 4, 0.0, 0, None, 0, None, None, None, 0, None) == -1
    # _ex entry points: unknown flag bits are rejected
    assert L.dstd_block_train_fwd_ex(None, None, 4, 35, 22, 0.1, None, None, 0, None, 1) == -1
    assert L.dstd_model_train_fwd_ex(None, None, 4, 0.1, 0.0, 0, None, None, 0, None, 4) == -1
    assert L.dstd_mpjpe_fwd(None, None, 10, None, None, 0, None) == -1
    assert L.dstd_frame_mpjpe(None, None, 1, 35, 96, 0, None, 66, None, None, 6, None, None) == -1


def test_version_and_errors():
    L = native.lib()
    assert b"gfx950" in L.dstd_version()
    # provenance: the loaded binary was built from exactly this tree's sources
    assert L.dstd_source_hash().decode() == native.source_hash()
    assert L.dstd_error_string(-2) == b"workspace too small"
    assert b"envelope" in L.dstd_error_string(-3)


def test_workspace_sizes_scale_with_batch():
    L = native.lib()
    a = L.dstd_model_workspace_bytes(1, 35, 22, 64, 5)
    b = L.dstd_model_workspace_bytes(256, 35, 22, 64, 5)
    assert 0 < a < b
    # three NTVC activations + adjacency scratch per sample dominate
    per = 3 * 35 * 22 * 64 * 4 + (2 * 35 * 22 * 22 + 22 * 35 * 35) * 4
    assert b >= 256 * per
    assert L.dstd_dstdgc_workspace_bytes(0, 4, 64, 64, 35, 22) > 0
    assert L.dstd_block_workspace_bytes(4, 6, 64, 35, 22) > 0


def test_capi_rejects_bad_arguments_without_gpu():
    L = native.lib()
    # null pointers are rejected before any device work
    assert L.dstd_model_fwd(None, None, 4, None, None, 0, None) == -1
    assert L.dstd_block_fwd(None, None, 4, 35, 22, None, None, 0, None) == -1
    w = native.GCWeights()
    assert L.dstd_dstdgc_fwd(0, None, 4, 64, 64, 35, 22, w, None, None, None, None, 0, None) == -1


def test_state_dict_schema_matches_reference():
    m = get_model("dstdgcn", dstdgcn=H36M)
    d = load_npz("model_h36m.npz")
    ref = [k[3:] for k in d.files if k.startswith("sd/")]
    assert list(m.state_dict().keys()) == ref
    for k in ref:
        assert tuple(m.state_dict()[k].shape) == d["sd/" + k].shape, k
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == 173999
    assert sum(p.numel() for p in m.parameters()) == 189350
    m.load_state_dict({k: torch.from_numpy(d["sd/" + k]) for k in ref})


def test_registry_keyerror():
    with pytest.raises(KeyError):
        get_model("stsgcn", stsgcn={})


def test_A_s_R_s_alias_like_reference():
    blk = DSTDGCB(64, 64, 35, 22, "h36m")
    assert blk.A_s.data_ptr() == blk.R_s.data_ptr()
    sd = blk.state_dict()
    sd["A_s"] = torch.zeros_like(sd["A_s"])
    sd["R_s"] = torch.full_like(sd["R_s"], 3.0)
    blk.load_state_dict(sd)
    assert torch.all(blk.A_s == 3.0) and torch.all(blk.R_s == 3.0)


def test_cpu_forward_fails_loudly():
    m = get_model("dstdgcn", dstdgcn=H36M).eval()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(2, 35, 22, 3))
    op = DSTDGC(64, 64, 35, 22, mode="spatial")
    with pytest.raises(RuntimeError):
        op(torch.zeros(1, 64, 35, 22), torch.zeros(1, 22, 22), 1.0)


def test_train_mode_on_cpu_fails_loudly():
    m = get_model("dstdgcn", dstdgcn=H36M).train()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(2, 35, 22, 3))
    blk = DSTDGCB(64, 64, 35, 22, "h36m").train()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        blk(torch.zeros(2, 64, 35, 22))


def test_library_exports_every_aux_header_symbol():
    L = native.lib()
    syms = header_symbols("dstd_gcn_aux.h")
    assert len(syms) == 6, syms
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(native.AUX_EXPORTS)
    assert L.dstd_ctg_fwd(None, 2, 8, 10, 22, None, None, None, None, None, 0, None) == -1
    assert L.dstd_conv2d_fwd(None, 2, 8, 10, 22, None, None, 8, 3, 1, 1, 1, 1, 0, None, None, 0, None) == -1


def test_plain_st_gcnn_layer_schema_matches_reference():
    """ST_GCNN_layer(refine=False) builds ConvTemporalGraphical + Conv2d with
    the reference's parameter names and shapes (plain_layers.npz state dicts)."""
    from model import ST_GCNN_layer
    d = load_npz("plain_layers.npz")
    for name, (cin, cout, ks, T) in {"p_64_32_k31": (64, 32, [3, 1], 35), "p_16_16_k33": (16, 16, [3, 3], 20),
                                     "p_8_12_k11": (8, 12, [1, 1], 10)}.items():
        layer = ST_GCNN_layer(cin, cout, ks, 1, T, 22, True, False, True, "h36m")
        ref = group(d, f"{name}/sd/")
        sd = layer.state_dict()
        assert list(sd.keys()) == list(ref.keys())
        for k in ref:
            assert tuple(sd[k].shape) == ref[k].shape, k
        assert np.array_equal(sd["stgcn.0.A_fixed"].numpy(), ref["stgcn.0.A_fixed"])
        layer.load_state_dict({k: torch.from_numpy(v) for k, v in ref.items()})


def test_torch_library_ops_and_fake_kernels():
    """The eval forwards are torch.library custom ops whose fake
    kernels give the output shapes without a GPU (meta tensors)."""
    for name in ("dstdgc_forward", "dstdgcb_forward", "dstdgcn_forward"):
        assert hasattr(torch.ops.dstd, name), name
    m = get_model("dstdgcn", dstdgcn=H36M)
    meta = [t.to("meta") for t in list(m.parameters()) + list(m.buffers())]
    y = torch.ops.dstd.dstdgcn_forward(torch.empty(3, 35, 22, 3, device="meta"), meta, m._dstd_uid, 0)
    assert y.shape == (3, 35, 22, 3) and y.device.type == "meta"
    blk = m.encoders[0][0].stgcn[0][0]
    out = m.conv_st_out.stgcn[0][0]
    tb = [t.to("meta") for t in list(out.parameters()) + list(out.buffers())]
    assert torch.ops.dstd.dstdgcb_forward(torch.empty(2, 64, 35, 22, device="meta"), tb, out._dstd_uid, 3,
                                          0).shape == (2, 3, 35, 22)
    op = blk.conv_s[0]
    w = [t.to("meta") for t in op.parameters()]
    assert torch.ops.dstd.dstdgc_forward(torch.empty(2, 64, 35, 22, device="meta"), torch.empty(22, 22, device="meta"),
                                         torch.empty(1, device="meta"), w, op._dstd_uid).shape == (2, 64, 35, 22)


def test_copies_get_their_own_instance_token():
    import copy
    m = get_model("dstdgcn", dstdgcn=H36M)
    c = copy.deepcopy(m)
    assert c._dstd_uid != m._dstd_uid
    assert c.encoders[0][0].stgcn[0][0]._dstd_uid != m.encoders[0][0].stgcn[0][0]._dstd_uid


def test_no_mixed_shape_mfma_chains_in_the_library():
    """The built library's gfx950 ISA holds no MFMA that accumulates onto the
    previous MFMA's result with a different MFMA shape within 5 wait states
    (dstd_hilo.h, "a gfx950 MFMA hazard hipcc does not pad"; reproducer
    scripts/micro/mfma_read_hazard.hip).  hipcc pads nothing there, so this is
    checked on the code object itself (scripts/mfma_hazard_audit.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import mfma_hazard_audit as A
    findings, n_mfma, n_funcs = A.audit(native.LIB_PATH)
    assert n_funcs > 100 and n_mfma > 10000  # every translation unit's code object was read
    assert not findings, findings[:5]
