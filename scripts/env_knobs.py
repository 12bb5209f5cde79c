"""HIP runtime knobs against the launch-bound legs (why
the graph replay is not faster than eager launches).  One process per knob
setting (the runtime reads them at initialisation): prints one JSON line with
the B=32 eval forward eager / graph-frozen, the B=256 forward and the B=32
training step eager / graphed, under the DEBUG_* / HIP_* variables of the
current environment.

usage: KNOB=VALUE python scripts/env_knobs.py [--label L] [--no-train]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import bench  # noqa: E402

KNOBS = ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "DEBUG_HIP_GRAPH_BATCH_SIZE", "DEBUG_HIP_FORCE_GRAPH_QUEUES",
         "DEBUG_CLR_KERNARG_HDP_FLUSH_WA", "HIP_FORCE_DEV_KERNARG", "DEBUG_HIP_KERNARG_COPY_OPT",
         "DEBUG_CLR_MAX_BATCH_SIZE", "ROC_USE_FGS_KERNARG")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--trace", choices=("eager", "graph"), help="only 100 B=32 forwards of one kind (for a kernel trace)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model, opts, _ = bench.load_model("h36m", dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    x = bench.synth_input(256, T, 22, opts["input_time_frame"], 1234).to(dev)
    if args.trace:
        xb = x[:32].contiguous()
        with torch.no_grad():
            fn = (lambda: model(xb)) if args.trace == "eager" else model.graphed(xb, frozen=True)
            for _ in range(10):
                fn() if args.trace == "eager" else fn(xb)
            torch.cuda.synchronize()
            for _ in range(100):
                fn() if args.trace == "eager" else fn(xb)
            torch.cuda.synchronize()
        return
    out = {"label": args.label, "env": {k: os.environ[k] for k in KNOBS if k in os.environ}}
    sb = bench.small_batch_leg(model, x, 32, args.steps, 20)
    out["b32_eager_ms"] = sb["ms_per_step"]
    out["b32_host_us"] = sb["host_us_per_call"]
    out["b32_graph_ms"] = sb["graph_replay_frozen"]["ms_per_step"]
    out["b32_graph_host_us"] = sb["graph_replay_frozen"]["host_us_per_call"]
    with torch.no_grad():
        ms, host = bench.timed_calls(lambda: model(x), args.steps // 2, 10)
    out["b256_ms"] = round(ms, 4)
    if not args.no_train:
        tr = bench.train_leg(dev, 32, 30, 5)
        out["train_ms"] = tr["ms_per_step"]
        out["train_issue_us"] = tr["host_issue_us_per_step"]
        out["train_graph_ms"] = tr["graph_replay"]["ms_per_step"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
