"""Probe: one B=256 H36M forward as S concurrent half / quarter batches on S
HIP streams (one model instance per stream: each owns its workspace), the
block kernel forced at the smaller per-stream batch (DSTD_FWD_FUSED_TEMPORAL).
The launches of different streams overlap each other's fill / drain and
desynchronise the phases of their workgroups (phase 3's plane-store burst of
one stream against the LDS-bound phases of the other).  Interleaved rounds,
wall ms per 256 sequences; outputs checked bit-identical to the one-stream
forward.

  python scripts/stream_split_probe.py [--config h36m] [--rounds 5] [--steps 20]
"""
import argparse
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
import bench  # noqa: E402
import dstd_native as native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="h36m")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--splits", default="1,2,4")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model, opts, _ = bench.load_model(args.config, dev)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = {"h36m": 22, "cmu": 25, "3dpw": 23}[args.config]
    B = 256
    x = bench.synth_input(B, T, V, opts["input_time_frame"], 3).to(dev)
    splits = [int(s) for s in args.splits.split(",")]
    cfgs = {}
    for S in splits:
        if S == 1:
            cfgs[S] = ([model], [torch.cuda.current_stream()])
            continue
        ms = []
        for _ in range(S):
            m = copy.deepcopy(model)
            m._dstd_fwd_flags = native.FWD_FUSED_TEMPORAL
            ms.append(m)
        cfgs[S] = (ms, [torch.cuda.Stream() for _ in range(S)])

    def run(S):
        ms, ss = cfgs[S]
        if S == 1:
            return ms[0](x)
        main = torch.cuda.current_stream()
        n = B // S
        outs = [None] * S
        for i in range(S):
            ss[i].wait_stream(main)
            with torch.cuda.stream(ss[i]):
                outs[i] = ms[i](x[i * n:(i + 1) * n])
        for i in range(S):
            main.wait_stream(ss[i])
        return torch.cat(outs)

    with torch.no_grad():
        ref = run(1)
        for S in splits:
            y = run(S)
            torch.cuda.synchronize()
            print(f"S={S}: bit-identical to one stream: {torch.equal(y, ref)}", flush=True)
        res = {S: [] for S in splits}
        for _ in range(args.rounds):
            for S in splits:
                for _ in range(3):
                    run(S)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.steps):
                    run(S)
                e1.record()
                torch.cuda.synchronize()
                res[S].append(e0.elapsed_time(e1) / args.steps)
        for S in splits:
            v = sorted(res[S])
            print(f"{args.config} S={S}: median {v[len(v) // 2]:.4f} ms (min {v[0]:.4f}) per 256-sequence forward")


if __name__ == "__main__":
    main()
