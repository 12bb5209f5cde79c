"""B=32 frozen-graph replay (DSTDGCN.graphed) against eager, by how the new
input reaches the graph's static input: torch copy_ (hipMemcpyAsync, a
rocclr blit), none (the caller writes run.input itself), or a gather kernel
(index_select, an ordinary kernel launch).  Prints ms per call for each,
interleaved rounds.  (the replay was slower than eager.)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
model, opts, _ = bench.load_model("h36m", dev)
T = opts["input_time_frame"] + opts["output_time_frame"]
x = bench.synth_input(256, T, 22, opts["input_time_frame"], 1234).to(dev)
xb = x[:32].contiguous()
res = {}
with torch.no_grad():
    gz = model.graphed(xb, frozen=True)
    y_eager = model(xb).clone()
    idx = torch.arange(xb.numel(), device=dev)
    flat_in = gz.input.view(-1)

    def gather(xn):
        torch.index_select(xn.view(-1), 0, idx, out=flat_in)
        return gz(gz.input)

    kinds = {"eager": lambda: model(xb), "graph_copy": lambda: gz(xb), "graph_nocopy": lambda: gz(gz.input),
             "graph_gather": lambda: gather(xb)}
    for k, f in kinds.items():
        assert torch.equal(f(), y_eager), k
    for r in range(3):
        for k, f in kinds.items():
            ms, host = bench.timed_calls(f, 300, 20)
            res.setdefault(k, []).append(round(ms, 4))
print(json.dumps(res))
