"""Host-side logic of the model drop-in (no GPU): the cached walk of the
module tree that replaces ``parameters()`` / ``buffers()`` on the hot path
(model/dstdgcn.py:_TensorTree) must always equal torch's own walk."""
import copy

import torch

from model import get_model

OPTS = dict(input_channels=6, input_time_frame=10, output_time_frame=25, st_gcnn_dropout=0.0,
            joints_to_consider=22, num_feature=64, num_layers=7, layout="h36m")


def same(m):
    p, b = m._tree.get(m)
    tp, tb = list(m.parameters()), list(m.buffers())
    return len(p) == len(tp) and len(b) == len(tb) and all(x is y for x, y in zip(p, tp)) and all(
        x is y for x, y in zip(b, tb))


def test_tensor_tree_matches_torch_walk_and_invalidates():
    m = get_model("dstdgcn", dstdgcn=OPTS)
    assert same(m) and same(m)  # built, then reused
    m.prelu.weight = torch.nn.Parameter(torch.ones(1))  # replaced parameter
    assert same(m)
    m.bn_in.bn.running_mean = torch.zeros_like(m.bn_in.bn.running_mean)  # replaced buffer
    assert same(m)
    m.encoders[0] = copy.deepcopy(m.encoders[0])  # replaced submodule
    assert same(m)
    m.encoders[1].register_parameter("extra", torch.nn.Parameter(torch.ones(2)))  # added parameter
    assert same(m)
    m.encoders[2].add_module("extra", torch.nn.Linear(2, 2))  # added submodule
    assert same(m)
    m2 = copy.deepcopy(m)
    assert same(m2)
    assert not any(x is y for x, y in zip(m2._tree.get(m2)[0], m.parameters()))


def test_tensor_tree_sees_functional_call_swaps():
    """torch.func.functional_call swaps tensors into _parameters / _buffers
    directly (no registration hook): inside the call the cached walk must hand
    out the swapped-in tensors, after it the module's own again."""
    m = get_model("dstdgcn", dstdgcn=OPTS)
    assert same(m)
    own = m._tree.get(m)[0]
    new = {k: v.detach().clone() for k, v in m.named_parameters()}
    seen = {}

    def probe(self, x):
        seen["params"] = list(self._tree.get(self)[0])
        seen["same"] = same(self)
        return x

    orig = type(m).forward
    type(m).forward = probe
    try:
        torch.func.functional_call(m, new, (torch.zeros(1),))
    finally:
        type(m).forward = orig
    assert seen["same"]
    assert all(a is b for a, b in zip(seen["params"], new.values()))
    assert same(m) and all(a is b for a, b in zip(m._tree.get(m)[0], own))


def test_fast_variant_schema_and_derivation_cpu():
    """model.dstdgcn_fast (reference model/dstdgcn_fast.py): the reference's
    state_dict keys in order, and the dstdgcn.py-schema shadow derived from
    it (m1/m2 swapped, -W_rm, A^T, Linear -> 1x1 conv, BN (v,c) -> (c,v))
    reproduces the reference's fp64 output through the dstdgcn.py oracle;
    building the shadow leaves the caller's RNG alone."""
    import numpy as np

    from conftest import group, load_npz
    from model import dstdgcn_fast as F
    from oracle import dstdgcn_oracle as O

    d = load_npz("dstdgcn_fast.npz")
    for tag in ("h36m", "3dpw"):
        p = f"model_{tag}/"
        sd = group(d, p + "sd/")
        opts = {k[len(p + "opt/"):]: d[k].item() for k in d.files if k.startswith(p + "opt/")}
        m = F.DSTDGCN(**opts)
        assert list(m.state_dict()) == list(sd)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        state = torch.random.get_rng_state()
        sh = m._shadow_for(torch.device("cpu"))
        assert torch.equal(state, torch.random.get_rng_state())
        m._sync(sh)
        y = O.dstdgcn(d[p + "x"], {k: v.detach() for k, v in sh.state_dict().items()}, opts["num_layers"])
        ref = d[p + "y64"]
        assert np.abs(y.numpy() - ref).max() / np.abs(ref).max() < 1e-6
        assert not any(k.startswith("_shadow") for k in m.state_dict())
        c = copy.deepcopy(m)
        assert c.__dict__["_shadow"] is None


def test_anchor_of_selects_the_parameter_inputs():
    """The training Function's parameter inputs (model/dstdgcn.py:_anchor_of):
    one empty leaf requiring grad only in the opted-in in-place gradient mode
    (engine.PredictionEngine.train) with grad enabled, a plain tensor and no
    parameter hooks -- otherwise the parameters themselves, so hooks, DDP and
    torch.autograd.grad keep ordinary autograd gradients."""
    from model.dstdgcn import _anchor_of
    m = get_model("dstdgcn", dstdgcn=OPTS)
    params = m._tree.get(m)[0]
    x = torch.zeros(2, 35, 22, 3)
    assert _anchor_of(m, x, params) is params  # default: not opted in
    m._dstd_inplace_grads = True
    a = _anchor_of(m, x, params)
    assert len(a) == 1 and a[0].requires_grad and a[0].numel() == 0 and a[0].is_leaf
    assert _anchor_of(m, x, params)[0] is a[0]  # one leaf per model
    with torch.no_grad():
        assert _anchor_of(m, x, params) is params
    h = next(p for p in params if p.requires_grad).register_hook(lambda g: g)
    assert _anchor_of(m, x, params) is params  # a hook: parameter inputs
    h.remove()
    assert _anchor_of(m, x, params)[0] is a[0]
    frozen = [p.detach() for p in params]  # nothing requires grad: parameter inputs
    assert _anchor_of(m, x, frozen) is frozen
