"""Host-side checks of the engine counterpart: the
test-metric index tables and checkpoint I/O, no GPU needed (the metric and
loss kernels themselves are covered by tests/test_gpu_train.py)."""
import os

import numpy as np
import pytest
import torch

from conftest import group, load_npz
from engine import AccumLoss, ModelWrapper, PredictionEngine, tsc_inverse, tsc_transform
from model import get_model
from oracle import dstdgcn_oracle as O

H36M = dict(input_channels=6, input_time_frame=10, output_time_frame=25, st_gcnn_dropout=0.1,
            joints_to_consider=22, num_feature=64, num_layers=5, layout="h36m")
CFG = dict(learn=dict(opt="adam", lr=3e-3, weight_decay=0, gamma=0.9, step_size=5),
           loss=dict(joint=["jl2", 1]), n_out=1, transform="tsc", use_weight=False, inverse=True)


class _Log:
    def __init__(self):
        self.lines = []

    def info(self, msg, *a, **k):
        self.lines.append(msg)


def _engine(model=None):
    return PredictionEngine(CFG, model if model is not None else get_model("dstdgcn", dstdgcn=H36M), _Log())


def test_tsc_views():
    x = torch.arange(2 * 3 * 12.).view(2, 3, 12)
    y = tsc_transform(x)
    assert y.shape == (2, 3, 4, 3) and y.data_ptr() == x.data_ptr()
    assert torch.equal(tsc_inverse(y), x)


def test_accum_loss_like_reference():
    a = AccumLoss()
    a.update(3.0, 2)
    a.update(5.0, 2)
    assert a.avg == 2.0 and a.val_his == [3.0, 5.0]


def test_unbuilt_losses_and_transforms_raise():
    m = get_model("dstdgcn", dstdgcn=H36M)
    with pytest.raises(NotImplementedError):
        ModelWrapper(m, {"bone": ["bl2", 1]})
    with pytest.raises(NotImplementedError):
        PredictionEngine(dict(CFG, transform="tscr_h36m"), m, _Log())


def test_metric_index_tables_reproduce_reference_fill():
    """used_pos / joint_src (what dstd_frame_mpjpe reads) rebuild the
    reference's pred_3d (prediction.py:369-389) exactly."""
    d = load_npz("engine.npz")
    eng = _engine()
    all_seqs = torch.from_numpy(d["test/all_seqs"])
    n, T, D = all_seqs.shape
    outputs = torch.randn(n, T, len(d["test/dim_used"]))
    used_pos, joint_src, frames = eng._metric_indices(D, outputs.shape[2], T, 10, list(d["test/eval_frame"]),
                                                      d["test/dim_used"], d["test/joint_to_ignore"],
                                                      d["test/joint_equal"])
    assert frames.tolist() == [10 + f for f in d["test/eval_frame"]]
    pred = PredictionEngine._fill_pred(all_seqs, outputs, used_pos, joint_src, 0)
    ref = all_seqs.clone().numpy()
    ref[:, :, d["test/dim_used"]] = outputs.numpy()
    ji, je = d["test/joint_to_ignore"], d["test/joint_equal"]
    ref[:, :, np.concatenate((ji * 3, ji * 3 + 1, ji * 3 + 2))] = ref[:, :, np.concatenate((je * 3, je * 3 + 1,
                                                                                           je * 3 + 2))]
    assert np.array_equal(pred.reshape(n, T, D).numpy(), ref)
    # and the per-frame metric of that fill equals the oracle restatement
    m = O.test_metric(all_seqs.numpy(), outputs.numpy(), 10, d["test/eval_frame"], d["test/dim_used"], ji, je)
    p = pred.numpy().astype(np.float64)
    t = all_seqs.numpy().reshape(n, T, -1, 3).astype(np.float64)
    mine = np.array([np.linalg.norm(t[:, 10 + f] - p[:, 10 + f], axis=-1).mean() * n for f in d["test/eval_frame"]])
    assert np.allclose(mine, m, rtol=1e-12)


def test_checkpoint_roundtrip_and_reference_schema(tmp_path):
    """save/recover (prediction.py:159-182): the same dict, 'model.'-prefixed
    keys, loadable with weights_only=True, A_s/R_s alias kept on load."""
    d = load_npz("model_h36m.npz")
    m = get_model("dstdgcn", dstdgcn=H36M)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in group(d, "sd/").items()})
    eng = _engine(m)
    eng.save(str(tmp_path), err=12.5, epoch=7, is_best=True)
    assert os.path.exists(tmp_path / "last.pth") and os.path.exists(tmp_path / "best.pth")
    state = torch.load(tmp_path / "last.pth", weights_only=True)
    assert set(state) == {"lr", "err", "model", "optimizer", "scheduler", "epoch"}
    ref_keys = ["model." + k[3:] for k in d.files if k.startswith("sd/")]
    assert list(state["model"].keys()) == ref_keys
    assert len(ref_keys) == 309  # SURVEY §8(b) state schema
    fresh = _engine()
    epoch, err = fresh.recover(str(tmp_path / "last.pth"))
    assert (epoch, err) == (7, 12.5)
    for k, v in m.state_dict().items():
        assert torch.equal(fresh.model.model.state_dict()[k], v), k
    for blk in (fresh.model.model.conv_st_in.stgcn[0][0], fresh.model.model.encoders[2][0].stgcn[0][0]):
        assert blk.A_s.data_ptr() == blk.R_s.data_ptr()
    # a checkpoint written in the reference's format (plain dict, reference key
    # names under 'model.') loads the same way
    ref_state = {"lr": 3e-3, "err": 1.0, "epoch": 3, "model": {"model." + k[3:]: torch.from_numpy(d[k])
                                                                for k in d.files if k.startswith("sd/")},
                 "optimizer": fresh.optimizer.state_dict(), "scheduler": fresh.scheduler.state_dict()}
    torch.save(ref_state, tmp_path / "ref.pth")
    other = _engine()
    assert other.recover(str(tmp_path / "ref.pth")) == (3, 1.0)
    x = torch.from_numpy(d["x"])
    y = O.dstdgcn(x, {k: v for k, v in other.model.model.state_dict().items()}, 5)
    assert float((y - torch.from_numpy(d["y64"]).double()).abs().max()) < 1e-4 * float(np.abs(d["y64"]).max())
