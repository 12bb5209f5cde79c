"""A training step captured once as a HIP graph and replayed (SURVEY §8(f)
row 2: the engine's step, engine/prediction.py:231-294).

The native training path launches ~500 kernels per step (forward pair, two
losses, backward, Adam); eagerly the host spends ~5.6 ms issuing them for a
B=32 step whose kernels take less than half of that.  Captured with
``torch.cuda.CUDAGraph`` the step is one graph launch: the host cost
disappears and the kernels run back to back.

What makes the step capturable:
* every native launch goes to the current stream and allocates through the
  torch caching allocator (the graph's private pool during capture);
* the dropout seed is drawn on the device (DSTD_TRAIN_SEED_DEVICE), so each
  replay draws a fresh mask;
* the optimizer is ``torch.optim.Adam(..., capturable=True)`` with a tensor
  learning rate (StepLR updates it in place);
* the parameters' ``.grad`` are slices of the model's persistent gradient
  arena (dstd_native.grad_sink), installed during the warm-up and zeroed by a
  captured kernel at the start of every replay.

Capturing needs warm-up steps (lazy optimizer state, workspaces, the
arena); they run on the example batch and their effect on the parameters,
buffers and optimizer state is undone before the first replay, so replay k
is exactly eager step k.
"""
import torch

import dstd_native as native
from model.dstdgcn import invalidate_native_cache


def _opt_state_tensors(optimizer):
    out = []
    for group in optimizer.param_groups:
        for p in group["params"]:
            for k, v in optimizer.state.get(p, {}).items():
                if torch.is_tensor(v):
                    out.append((p, k, v))
    return out


class GraphedStep:
    """``step_fn(*args) -> tuple of tensors`` (e.g. the step's losses), run
    once per call; the arguments are copied into static device buffers of
    the example's shapes and the captured graph replays.  Call with tensors
    of the same shapes and dtypes as the example (a different shape is the
    caller's to run eagerly)."""

    def __init__(self, step_fn, example_args, model, optimizer, warmup=3):
        dev = example_args[0].device
        self.shapes = [(a.shape, a.dtype) for a in example_args]
        self.static = [a.detach().clone() for a in example_args]
        # state the warm-up will move: parameters, buffers, optimizer state
        snap_model = [t.detach().clone() for t in list(model.parameters()) + list(model.buffers())]
        before = {(id(p), k): v.detach().clone() for p, k, v in _opt_state_tensors(optimizer)}
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn(*self.static)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)  # a stream of its own: its workspace is private to this graph
        with torch.cuda.graph(self.graph, stream=cap):
            self.outputs = step_fn(*self.static)
        torch.cuda.synchronize(dev)
        # the capture's native workspace lives in the graph's memory pool: keep
        # it with the graph and out of the eager cache, where a later, larger
        # claim on the same stream would free it under the graph
        self._workspace = native._ws_cache.pop((str(dev), cap.cuda_stream), (None, None))[0]
        self.model = model
        # undo the warm-up: replay 1 is step 1
        with torch.no_grad():
            for t, s in zip(list(model.parameters()) + list(model.buffers()), snap_model):
                t.copy_(s)
            for p, k, v in _opt_state_tensors(optimizer):
                old = before.get((id(p), k))
                if old is None:  # created lazily by the warm-up (Adam: zeros, step 0)
                    v.zero_()
                else:
                    v.copy_(old)

    def matches(self, *args):
        return len(args) == len(self.shapes) and all(
            a.shape == s and a.dtype == d for a, (s, d) in zip(args, self.shapes))

    def __call__(self, *args):
        for dst, src in zip(self.static, args):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        # the replay updated parameters and BatchNorm buffers on the device
        # without moving their version counters: the next eval forward must
        # not reuse constants folded from the previous weights
        invalidate_native_cache(self.model)
        return self.outputs
