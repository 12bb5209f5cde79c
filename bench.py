#!/usr/bin/env python
"""Throughput of the MI355X DSTDGC hot path (BASELINE.json metric).

A "step" is one eval-mode DSTDGCN forward over one synthetic H36M-shape batch
(B=256 per GPU, T = 10 + 25 = 35 frames, V = 22 joints), inputs
already resident in HBM.  Weights are the committed H36M fixture state dict
(tests/golden/model_h36m.npz: random init, dynamic terms randomised, BN
calibrated), so activations stay finite; values do not change the work.

  python bench.py [--gpus N --steps K --warmup W] [--global-batch G]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
         weak scaling (default): every rank runs its own B=256 shard;
         --global-batch G: strong scaling, G sequences split over the ranks
         (2048).  No data-path collective either way;
         the per-rank elapsed time is MAX-reduced over RCCL.

Timing: barrier + synchronize, t0, exactly K steps, synchronize, t1, barrier
(the barriers bracket the region but are not inside it).

One JSON line on rank 0.  Besides the driver's fields it carries
  roofline     : the dominant kernel family (largest summed time per step in
                 an untimed profiled pass; at B >= the CU count the block
                 kernel, one launch per DSTDGCB) and its launch in DSTDGCB 1
                 (the first encoder, a 64->64 split-f16 launch), bracketed by
                 two HIP events on the launch stream in one of every
                 --probe-every timed steps.  achieved = the launch's COMPULSORY
                 bytes (the block -- or, in the two-launch
                 schedule, each of its GCs -- reads its input and writes its
                 output once, 394,240 B per H36M sequence, x B sequences) / its
                 average duration, against the 8 TB/s HBM3E peak.  layout_bytes: what the
                 launch moves by design in this build's stored layouts (the
                 adjacency planes and P/Q it reads on top).  traffic: measured HBM
                 bytes per launch of that kernel (profiles/pmc_traffic.json,
                 rocprofv3 PMC passes).  whole_forward: compulsory bytes of the
                 whole forward (2.393 MB per H36M sequence, each block's input
                 read and output written once) and FLOPs over the step time.
  cpu_baseline : the CPU oracle (op-for-op restatement of the reference
                 forward, torch fp32) timed on this host's cores, N=1 only; the
                 thread-count sweep is on the line, the best count is `value`.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dstd-gcn_amd"))
sys.path.insert(0, ROOT)

import dstd_dist as D  # noqa: E402
import dstd_native as native  # noqa: E402
from model import get_model  # noqa: E402

METRIC = "pose-sequences/sec forward (H36M 22J×50T, B=256) at 1/2/4/8 GPUs; % HBM roofline"
PEAK_FP32_TFLOPS = 157.3   # MI355X fp32 MFMA / vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
PEAK_F16_DENSE_TFLOPS = 2500.0  # MI355X dense f16 MFMA (MI355X_MICROARCH.md); split-f16 runs 3 products per MAC

CONFIGS = {
    "h36m": ("model_h36m.npz", "H36M-shape synthetic, T=10+25=35, V=22"),
    "h36m75": ("model_h36m75.npz", "H36M-shape synthetic '50 in / 25 out', T=75, V=22"),
    "cmu": ("model_cmu.npz", "CMU-shape synthetic, T=35, V=25"),
    "3dpw": ("model_3dpw.npz", "3DPW-shape synthetic, T=40, V=23"),
}


def load_model(cfg, device):
    d = np.load(os.path.join(ROOT, "tests", "golden", CONFIGS[cfg][0]), allow_pickle=False)
    opts = {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}
    sd = {k[3:]: d[k] for k in d.files if k.startswith("sd/")}
    m = get_model("dstdgcn", dstdgcn=opts)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.to(device).eval(), opts, sd


def synth_input(B, T, V, Tin, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, V, 3, generator=g)
    x[:, Tin:] = x[:, Tin - 1:Tin]  # future frames = last observed (dataset/h36m.py:53-64)
    return x


# ---------------------------------------------------------------------------
# algorithmic FLOPs per sample of each kernel family
# ---------------------------------------------------------------------------
def block_flops(cin, cout, T, V, tail):
    TV, R = T * V, 2
    adj_s = 2 * (2 * R * T * V * V + 2 * T * (R * T) * V * V + T * V * V + 2 * T * V * V)
    spatial = 2 * (2 * cout * cin * TV + cout * TV) + 2 * (2 * cout * TV * V) + cout * TV + 4 * cout * TV
    if cin != cout:
        spatial += 2 * cout * cin * TV + cout * TV + 2 * cout * TV
    spatial += 2 * R * (2 * cout * TV + TV)  # P_t, Q_t of h (conv_m1/m2 of the temporal DSTDGC)
    adj_t = 2 * R * V * T * T + 2 * V * (R * V) * T * T + V * T * T + 2 * V * T * T
    temporal = 2 * cout * cout * TV + cout * TV + 2 * cout * T * T * V
    temporal += {"enc": 4, "in": 3, "out": 1}[tail] * cout * TV
    if tail != "out":
        temporal += 2 * 2 * R * (2 * cout * TV + TV)  # next block's P_s, Q_s
    return {native.KIND_ADJ_S: adj_s, native.KIND_SPATIAL: spatial, native.KIND_ADJ_T: adj_t,
            native.KIND_TEMPORAL: temporal}


def hl_sl_spatial(V):
    return 8 * ((V + 7) // 8)


def hl_sl_temporal(T):
    g = 0
    for s in range((T + 31) // 32):
        n = 0
        for kg in range(4):
            for e in range(8):
                if 32 * s + 16 * (e >> 2) + 4 * kg + (e & 3) < T:
                    n = kg + 1
        g += n
    return 8 * g


FUSED_TEMPORAL = {(35, 22), (35, 25), (40, 23)}  # dstd_hilo.hip temporal_fused_supported


def block_bytes(cin, cout, T, V, tail, split):
    """Layout bytes per sample of each kernel family of one DSTDGCB: what the
    launches move by design -- inputs read once, outputs written once, in the
    stored layouts (NTVC fp32 activations, channel-innermost P/Q, adjacencies
    as fp32 rows or split-f16 planes).  split: (spatial,
    temporal) launches run the split-f16 kernels; the split temporal launch of
    a FUSED_TEMPORAL shape builds its adjacency in LDS (no adjacency bytes)."""
    TV = T * V
    fused = split[1] and (T, V) in FUSED_TEMPORAL
    adj_s = 2 * T * (2 * V * hl_sl_spatial(V) * 2 if split[0] else 4 * ((V * V + 3) // 4 * 4))
    adj_t = 0 if fused else V * (2 * T * hl_sl_temporal(T) * 2 if split[1] else 4 * ((T * T + 3) // 4 * 4))
    pq_s, pq_t = TV * 8 * 4, TV * 4 * 4
    spatial = TV * cin * 4 + adj_s + TV * cout * 4 + pq_t
    temporal = TV * cout * 4 + adj_t + (TV * cout * 4 if tail == "enc" else 0) + TV * (cout if tail != "out" else 3) * 4
    if tail == "out":
        temporal += V * 3 * 4  # last observed frame of the model input
    else:
        temporal += pq_s
    if fused:  # the temporal launch reads the temporal P/Q itself
        return {native.KIND_ADJ_S: pq_s + adj_s, native.KIND_SPATIAL: spatial, native.KIND_ADJ_T: 0,
                native.KIND_TEMPORAL: temporal + pq_t}
    return {native.KIND_ADJ_S: pq_s + adj_s, native.KIND_SPATIAL: spatial, native.KIND_ADJ_T: pq_t + adj_t,
            native.KIND_TEMPORAL: temporal}


def op_compulsory_bytes(cin, cout, T, V):
    """one DSTDGC reads its input and writes its output once
    (fp32; weights excluded)."""
    return T * V * (cin + cout) * 4


def model_compulsory_bytes(opts):
    """per sequence, every DSTDGCB reads its input activation and
    writes its output once (fp32): 2.393 MB for H36M T=35 V=22."""
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V, C, L = opts["joints_to_consider"], opts["num_feature"], opts["num_layers"]
    cin0, cout_last = opts["input_channels"], opts["input_channels"] // 2
    return sum(T * V * (a + b) * 4 for a, b in [(cin0, C)] + [(C, C)] * L + [(C, cout_last)])


def phase3_moves(blocks, opts, split_on):
    """Blocks 1.. of a split forward at a FUSED_TEMPORAL shape get their
    spatial adjacency from the previous block's fused temporal launch
    (k_temporal_fused phase 3): that family's work moves there."""
    T = opts["input_time_frame"] + opts["output_time_frame"]
    if split_on and (T, opts["joints_to_consider"]) in FUSED_TEMPORAL:
        for i in range(len(blocks) - 1):
            blocks[i][native.KIND_TEMPORAL] += blocks[i + 1][native.KIND_ADJ_S]
            blocks[i + 1][native.KIND_ADJ_S] = 0
    return blocks


def model_block_bytes(opts, split_on):
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V, C, L = opts["joints_to_consider"], opts["num_feature"], opts["num_layers"]
    cin0, cout_last = opts["input_channels"], opts["input_channels"] // 2
    spec = [(cin0, C, "in")] + [(C, C, "enc")] * L + [(C, cout_last, "out")]
    out = []
    for cin, cout, tail in spec:
        split = (split_on and cin == 64 and cout == 64, split_on and cout == 64)
        out.append(block_bytes(cin, cout, T, V, tail, split))
    return phase3_moves(out, opts, split_on)


def merge_blocks(blocks, fused_t):
    """Each block as ONE launch (k_block_fused, the default wherever the fused
    temporal kernel runs): its spatial GC, its temporal adjacency (built in
    LDS) and its temporal GC (with phase 3) are one family, KIND_BLOCK; block
    0's spatial adjacency (built from the model input inside its launch,
    phase 0) too -- the later blocks' moved into the previous launch
    (phase3_moves) and are 0 here."""
    out = []
    for b in blocks:
        b = dict(b)
        b[native.KIND_BLOCK] = b.pop(native.KIND_SPATIAL) + b.pop(native.KIND_TEMPORAL) + \
            (b.pop(native.KIND_ADJ_T) if fused_t else 0) + b.pop(native.KIND_ADJ_S, 0)
        out.append(b)
    return out


def model_block_flops(opts, split_on=False):
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V, C, L = opts["joints_to_consider"], opts["num_feature"], opts["num_layers"]
    blocks = [block_flops(opts["input_channels"], C, T, V, "in")]
    blocks += [block_flops(C, C, T, V, "enc") for _ in range(L)]
    blocks.append(block_flops(C, opts["input_channels"] // 2, T, V, "out"))
    return phase3_moves(blocks, opts, split_on)


class Profiler:
    """Event pairs around the launches of chosen kernel families."""

    def __init__(self, L, pairs, kind_mask):
        self.L = L
        self.n = 2 * pairs
        self.events = (ctypes.c_void_p * self.n)()
        native.check(L.dstd_events_create(self.n, self.events), "dstd_events_create")
        self.kinds = (ctypes.c_int * pairs)()
        self.block = (ctypes.c_int * pairs)()
        self.prof = native.Profile(kind_mask, pairs, 0, self.events, self.kinds, self.block, -1)

    def elapsed(self):
        out = []
        ms = ctypes.c_float()
        for i in range(self.prof.count):
            native.check(self.L.dstd_event_elapsed_ms(self.events[2 * i], self.events[2 * i + 1], ctypes.byref(ms)),
                         "dstd_event_elapsed_ms")
            out.append((self.kinds[i], self.block[i], ms.value))
        return out

    def close(self):
        self.L.dstd_events_destroy(self.n, self.events)


def forward_profiled(model, x, y, prof):
    """The model's own eval forward (DSTDGCN._forward_native: constants reused
    across steps as in production) with event brackets."""
    model._forward_native(x, y, ctypes.byref(prof.prof))


def load_traffic(kernel, instance=None):
    """Measured HBM bytes per launch (profiles/pmc_traffic.json): the exact
    kernel instantiation when profiled, else the family average."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if instance and instance in d.get("by_kernel", {}):
            return d["by_kernel"][instance].get("hbm_bytes_per_launch")
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def split_instance(kind, T, V):
    """Kernel instantiation of DSTDGCB 1 (an encoder) for kind."""
    temporal = f"k_temporal_fused<{T}, {V}, 1, 64>" if (T, V) in FUSED_TEMPORAL else f"k_temporal_hl<{T}, 1, 64>"
    return {native.KIND_SPATIAL: f"k_spatial_hl<{V}, 64, 64>", native.KIND_TEMPORAL: temporal,
            native.KIND_BLOCK: f"k_block_fused<{T}, {V}, 64, 64, 1>",
            native.KIND_ADJ_S: f"k_adj_hl<0, {T}, {2 * T}, {V}>", native.KIND_ADJ_T: f"k_adj_hl<1, {V}, {2 * V}, {T}>"}.get(kind)


def cpu_baseline(opts, sd, x_cpu, min_s, max_s):
    """The fp32 CPU oracle on this host, on the bench's own B=256 batch: one
    forward per thread count (1, 16, 32, 64), then the best count timed for
    ~min_s seconds (`value`).  os.cpu_count() threads (256 on the MI355X box)
    is left out of the default run: it measured 0.8 seq/s (80 s per B=64
    forward; torch's intra-op pool on these small ops, profiles/r02_bench.json)."""
    from oracle import dstdgcn_oracle as O  # baseline leg only
    sd32 = {k: torch.from_numpy(v).float() for k, v in sd.items()}
    ncpu = os.cpu_count() or 1

    def fwd(xs):
        O.dstdgcn(xs, sd32, opts["num_layers"], dtype=torch.float32)

    sweep = {}
    with torch.no_grad():
        for th in sorted({1, min(16, ncpu), min(32, ncpu), min(64, ncpu)}):
            torch.set_num_threads(th)
            fwd(x_cpu[:8])  # warm-up at this count
            t0 = time.perf_counter()
            fwd(x_cpu)
            sweep[th] = round(x_cpu.shape[0] / (time.perf_counter() - t0), 1)
        best = max(sweep, key=sweep.get)
        torch.set_num_threads(best)
        n, t0 = 0, time.perf_counter()
        while True:
            fwd(x_cpu)
            n += 1
            el = time.perf_counter() - t0
            if el >= min_s or el >= max_s:
                break
    torch.set_num_threads(min(16, ncpu))
    return {"value": n * x_cpu.shape[0] / el, "unit": "seq/s", "cores": best, "kind": "port",
            "sample": f"{n} x B={x_cpu.shape[0]} forwards of the fp32 CPU oracle (oracle/dstdgcn_oracle.py, "
                      f"op-for-op restatement of model/dstdgcn.py:293-317), {el:.1f} s, torch {torch.__version__} "
                      f"CPU, {best} threads (the best of the sweep)",
            "thread_sweep_seq_s": sweep, "sweep_sample": f"one B={x_cpu.shape[0]} forward per thread count",
            "nproc": ncpu, "cpu_model": cpu_model()}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def config_leg(config, B, device, steps, warmup, cpu_seconds=None):
    """Side measurement at N=1 (not `value`): the eval forward of another
    BASELINE.json config through the drop-in call model(x), fixture weights of
    that layout.  "h36m75": BASELINE.json's metric names "22J x 50T" while the
    shipped yaml (dstdgcn_h36m.yaml:137-138) runs 10 + 25 frames, so the
    '50 in / 25 out' T=75 variant is on the line too; "cmu" / "3dpw": configs
    3 and the 3DPW shape at B=256.  cpu_seconds: the leg's own CPU baseline
    (the fp32 oracle on this host, same batch, same thread sweep as the main
    line's, BASELINE.md "Official CPU-baseline plan") and the GPU/CPU ratio."""
    model, opts, sd = load_model(config, device)
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    x_cpu = synth_input(B, T, V, opts["input_time_frame"], 1234)
    x = x_cpu.to(device)
    with torch.no_grad():
        ms, host = timed_calls(lambda: model(x), steps, max(warmup, 2))
    out = {"workload": CONFIGS[config][1] + f", B={B}, eval forward", "seq_len": T, "joints": V,
           "value": round(B / ms * 1e3, 2), "unit": "seq/s", "ms_per_step": round(ms, 4),
           "host_us_per_call": round(host, 2), "timed_call": "model(x)"}
    if cpu_seconds is not None:
        out["cpu_baseline"] = cpu_baseline(opts, sd, x_cpu, cpu_seconds, 30.0)
        out["vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    return out


def timed_calls(fn, steps, warmup):
    """(ms per call on the device clock, host us per call): fn() `steps` times
    between two synchronisations, after `warmup` untimed calls."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        fn()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, host / steps * 1e6


def arithmetic_leg(model, x, arith, steps, warmup):
    """Side measurement (not `value`): the same B=256 drop-in forward with the
    graph convolutions in another arithmetic (DSTDGCN.set_gc_arithmetic;
    "fp32" = exact-fp32 MFMA v_mfma_f32_16x16x4_f32 everywhere)."""
    prev = model.gc_arithmetic
    model.set_gc_arithmetic(arith)
    try:
        with torch.no_grad():
            ms, host = timed_calls(lambda: model(x), steps, warmup)
    finally:
        model.set_gc_arithmetic(prev)
    B = x.shape[0]
    return {"workload": f"same as the line, gc arithmetic {arith}", "value": round(B / ms * 1e3, 2), "unit": "seq/s",
            "ms_per_step": round(ms, 4), "host_us_per_call": round(host, 2)}


def small_batch_leg(model, x, B, steps, warmup):
    """Side measurement: eval throughput at the reference's test batch
    (dstdgcn_h36m.yaml:19 test_batch_size 32) through model(x), and the same
    forward replayed from a captured HIP graph (DSTDGCN.graphed)."""
    xb = x[:B].contiguous()
    with torch.no_grad():
        ms, host = timed_calls(lambda: model(xb), steps, warmup)
        out = {"workload": f"H36M-shape synthetic, B={B} (test_batch_size), eval forward", "value": round(B / ms * 1e3, 2),
               "unit": "seq/s", "ms_per_step": round(ms, 4), "host_us_per_call": round(host, 2)}
        if hasattr(model, "graphed"):
            g = model.graphed(xb)
            gms, ghost = timed_calls(lambda: g(xb), steps, warmup)
            out["graph_replay"] = {"value": round(B / gms * 1e3, 2), "ms_per_step": round(gms, 4),
                                   "host_us_per_call": round(ghost, 2), "note": "refolds the constants per replay"}
            gz = model.graphed(xb, frozen=True)
            gms, ghost = timed_calls(lambda: gz(xb), steps, warmup)
            out["graph_replay_frozen"] = {"value": round(B / gms * 1e3, 2), "ms_per_step": round(gms, 4),
                                          "host_us_per_call": round(ghost, 2),
                                          "note": "frozen weights: the GC launches alone after the first replay"}
    return out


def train_leg(device, B, steps, warmup):
    """Side measurement, SURVEY §8(d) config 5 on one GPU: one training step of
    the 3DPW model (T = 10 + 30, V = 23; dstdgcn_3dpw.yaml) = the engine's
    step (engine/prediction.py:231-294): train-mode forward of the batch and
    its time reversal (DSTDGCN.forward_pair), two mpjpe losses, native
    backward, Adam.  Random-init weights, synthetic poses."""
    from engine import mpjpe_error_3d
    opts = dict(input_channels=6, input_time_frame=10, output_time_frame=30, st_gcnn_dropout=0.0,
                joints_to_consider=23, num_feature=64, num_layers=5, layout="3dpw")
    torch.manual_seed(0)
    m = get_model("dstdgcn", dstdgcn=opts).to(device).train()
    m._dstd_inplace_grads = True  # as engine.PredictionEngine.train opts in
    opt = torch.optim.Adam(m.parameters(), lr=3e-3, fused=True)  # the engine's optimizer (eager steps)
    g = torch.Generator().manual_seed(1234)
    seq = torch.randn(B, 40, 69, generator=g)
    inp = seq.clone()
    inp[:, 10:] = inp[:, 9:10]
    inv = seq.flip(1).clone()
    inv[:, 10:] = inv[:, 9:10]
    seq, inp, inv = seq.to(device), inp.to(device), inv.to(device)
    seq_inv = seq.flip(1).contiguous()

    def step():
        out, out_i = m.forward_pair(inp.view(B, 40, 23, 3), inv.view(B, 40, 23, 3))
        loss = (mpjpe_error_3d(out.reshape(B, 40, 69), seq) + mpjpe_error_3d(out_i.reshape(B, 40, 69), seq_inv)) / 2
        opt.zero_grad()
        loss.backward()
        opt.step()

    ms, host = timed_calls(step, steps, warmup)
    # host_us_per_step above is the host's time per step in a back-to-back run,
    # which includes waiting for a full launch queue when the device is behind;
    # the cost of issuing one step is its host time from an idle queue
    issue = []
    for _ in range(7):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        step()
        issue.append((time.perf_counter() - h0) * 1e6)
    torch.cuda.synchronize()
    out = {"workload": f"3DPW-shape synthetic T=40 V=23, B={B}: forward pair + 2 mpjpe + backward + Adam (fp32)",
           "value": round(B / ms * 1e3, 2), "unit": "train seq/s", "ms_per_step": round(ms, 4),
           "host_us_per_step": round(host, 2), "host_issue_us_per_step": round(sorted(issue)[3], 2)}
    # the same step captured as one HIP graph (engine/graphed.py; what
    # PredictionEngine runs with learn.graph): capturable Adam, tensor lr
    from engine.graphed import GraphedStep
    torch.manual_seed(0)
    m2 = get_model("dstdgcn", dstdgcn=opts).to(device).train()
    m2._dstd_inplace_grads = True
    opt2 = torch.optim.Adam(m2.parameters(), lr=torch.tensor(3e-3, device=device), capturable=True)

    def step2(a, b, s, si):
        out2, out2_i = m2.forward_pair(a.view(B, 40, 23, 3), b.view(B, 40, 23, 3))
        loss2 = (mpjpe_error_3d(out2.reshape(B, 40, 69), s) + mpjpe_error_3d(out2_i.reshape(B, 40, 69), si)) / 2
        opt2.zero_grad()
        loss2.backward()
        opt2.step()
        return (loss2.detach(),)

    g = GraphedStep(step2, (inp, inv, seq, seq_inv), m2, opt2)
    gms, ghost = timed_calls(lambda: g(inp, inv, seq, seq_inv), steps, warmup)
    out["graph_replay"] = {"value": round(B / gms * 1e3, 2), "ms_per_step": round(gms, 4),
                           "host_us_per_step": round(ghost, 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="after the W warm-up steps, untimed forwards for this long so the timed region "
                         "starts at the GPU's steady clocks (a fresh box's first process otherwise reads "
                         "~1.5%% slow at K=20: profiles/r06ae_*); 0: off")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many sequences in total, split over the ranks")
    ap.add_argument("--config", default="h36m", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--side-cpu-seconds", type=float, default=3.0,
                    help="timed CPU oracle seconds (after the thread sweep) of each side config leg's own CPU baseline")
    ap.add_argument("--no-variant", action="store_true",
                    help="skip the side measurements of the other configs at N=1 (H36M '50 in / 25 out' T=75, "
                         "CMU and 3DPW at B=256)")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the N=1 side legs (exact fp32, B=32 eval, B=32 3DPW training step)")
    ap.add_argument("--probe-every", type=int, default=5,
                    help="bracket the dominant launch with HIP events in one of every P timed steps "
                         "(an event pair costs ~5%% of a step)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    host_group = None  # the group of the steps before and around the timed region
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:  # any torch.distributed.run launch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # The default group is RCCL, its communicator created at its first
        # collective: the elapsed-time MAX and the checksum exchange AFTER the
        # timed region.  A live RCCL communicator makes this forward's kernels
        # run 3-4% slower on this stack (gloo under torchrun does not;
        # profiles/r06y_*, r06z_*), so the weight broadcast and
        # the barriers around the timed region go over a gloo group (host-
        # staged; the forward itself has no collective).  Diagnostics:
        # DSTD_BENCH_RCCL_EARLY=1 (RCCL bound to the device at init and used
        # for everything, as before round 6), DSTD_BENCH_BACKEND=gloo.
        backend = os.environ.get("DSTD_BENCH_BACKEND", "nccl")
        early = backend == "nccl" and os.environ.get("DSTD_BENCH_RCCL_EARLY", "0") == "1"
        if early:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            host_group = dist.new_group(backend="gloo") if backend == "nccl" else None
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    model, opts, sd = load_model(args.config, device)
    if dist is not None:
        D.broadcast_module(model, src=0, group=host_group)  # weights once, rank 0 -> all
    T = opts["input_time_frame"] + opts["output_time_frame"]
    V = opts["joints_to_consider"]
    strong = args.global_batch > 0
    G = args.global_batch if strong else args.batch * world
    # one global batch, contiguous shard per rank (dstd_dist.shard_bounds)
    x_cpu = D.shard(synth_input(G, T, V, opts["input_time_frame"], 1234), world, rank).contiguous()
    B = x_cpu.shape[0]
    x = x_cpu.to(device)
    y = torch.empty_like(x)
    L = native.lib()
    fl = model_block_flops(opts, model.gc_arithmetic == "split")

    def barrier():
        if dist is not None:
            dist.barrier(group=host_group)

    with torch.no_grad():
        for _ in range(args.warmup):
            model(x)
        torch.cuda.synchronize()
        settle_steps = 0
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
            for _ in range(10):
                model(x)
            torch.cuda.synchronize()
            settle_steps += 10

        # untimed pass: per-family launch times -> dominant family
        nb = len(fl)
        prof = Profiler(L, args.steps * (2 + 4 * nb), (1 << len(native.KIND_NAMES)) - 1)
        for _ in range(args.steps):
            forward_profiled(model, x, y, prof)
        torch.cuda.synchronize()
        per_kind = {}
        for kind, _, ms in prof.elapsed():
            per_kind[kind] = per_kind.get(kind, 0.0) + ms
        prof.close()
        split_on = model.gc_arithmetic == "split"
        fused_t = split_on and (T, V) in FUSED_TEMPORAL
        fused_b = native.KIND_BLOCK in per_kind  # the blocks ran as single launches (k_block_fused)
        if fused_b:
            fl = merge_blocks(fl, fused_t)
        dominant = max((k for k in per_kind if k in fl[0]), key=lambda k: per_kind[k])

        # timed region: exactly K steps; in one of every P steps two events
        # around the dominant family's launch in DSTDGCB 1 (an encoder) -- an
        # event pair in every step slows the whole step by ~5%
        every = max(1, args.probe_every)
        prof = Profiler(L, (args.steps + every - 1) // every, 1 << dominant)
        prof.prof.only_block = 1
        probe = ctypes.byref(prof.prof)
        host_s = 0.0
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            # the drop-in call itself (DSTDGCN.forward -> _forward_native -> the C
            # ABI); a probed step carries the event brackets through the module
            if i % every == 0:
                model._dstd_profile = probe
            h0 = time.perf_counter()
            y = model(x)
            host_s += time.perf_counter() - h0
            model._dstd_profile = None
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        barrier()
        launches = prof.elapsed()
        prof.close()

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # metric exchange over RCCL after the timed region: output checksum
        # partials (the forward itself has no exchange)
        D.reduce_partials(y.double().abs().sum().reshape(1), torch.tensor([B], device=device))

    bb = model_block_bytes(opts, split_on)
    if fused_b:
        bb = merge_blocks(bb, fused_t)
    kernel_ms = sum(ms for _, _, ms in launches)
    avg_launch_s = kernel_ms * 1e-3 / max(len(launches), 1)
    C = opts["num_feature"]
    # compulsory bytes of the probed launch: DSTDGCB 1 is a 64 -> 64 block; its
    # spatial / temporal GC launch is one DSTDGC's input read + output write
    comp = op_compulsory_bytes(C, C, T, V) * B
    achieved = comp / avg_launch_s / 1e9 if kernel_ms > 0 else 0.0
    kname = native.KIND_NAMES[dominant]
    split_blk = split_on and opts["num_layers"] > 0
    traffic = load_traffic(kname + "_split" if split_blk else kname, split_instance(dominant, T, V) if split_blk else None)
    total_flop_per_seq = sum(sum(b.values()) for b in fl)
    # algorithmic FLOPs of the probed launch (the fused temporal launch also
    # builds its own adjacency and, phase 3, the next block's spatial one:
    # those families' FLOPs count to it -- phase3_moves did the latter)
    launch_flop = fl[1][dominant] + (fl[1][native.KIND_ADJ_T] if fused_t and dominant == native.KIND_TEMPORAL else 0)
    flops = launch_flop * B / avg_launch_s / 1e12 if kernel_ms > 0 else 0.0
    whole_bytes = model_compulsory_bytes(opts) * G * args.steps / elapsed / 1e9

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(G * args.steps / elapsed, 2),
            "unit": "seq/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "steps": settle_steps,
                       "note": "untimed forwards after the warm-up, before the timed region (steady clocks)"},
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "arithmetic": ("split-f16 MFMA for every contraction of the forward (fp32 operands as f16 hi/lo pairs, "
                           "three v_mfma_f32_16x16x32_f16 per product, fp32 accumulate; fp32 storage, VALU and "
                           "epilogues)") if split_on
                          else "exact-fp32 MFMA (v_mfma_f32_16x16x4_f32)",
            "data": "synthetic (N(0,1) poses, future frames padded with the last observed; fixture weights)",
            "config": {"workload": CONFIGS[args.config][1] + (f", {G} sequences over {world} GPU(s)" if strong else
                                                              f", B={B}/GPU") + ", eval forward",
                       "global_batch": G, "seq_len": T, "joints": V, "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "kernel": kname + (" (split-f16, DSTDGCB 1)" if split_blk else " (DSTDGCB 1)"),
                         "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "compulsory_bytes_per_launch": comp,
                         "compulsory_basis": f"SURVEY §8(d): {op_compulsory_bytes(C, C, T, V)} B/seq (" +
                                             ("one 64->64 DSTDGCB, the launch's whole block" if fused_b else
                                              "one 64->64 DSTDGC") +
                                             f": input read + output written once) x {B} seq",
                         "layout_bytes_per_launch": int(bb[1][dominant] * B) if launches else None,
                         "launches": len(launches), "probe_every": every,
                         "avg_launch_us": round(avg_launch_s * 1e6, 2),
                         "compute": {"flop_per_launch": launch_flop * B, "achieved_tflops": round(flops, 2),
                                     "frac_fp32_peak": round(flops / PEAK_FP32_TFLOPS, 4),
                                     "frac_split_f16_ceiling": round(flops / (PEAK_F16_DENSE_TFLOPS / 3), 4),
                                     "note": "fp32 FLOPs of the launch over the fp32 peak (157 TF, SURVEY §8(d)) and "
                                             "over the split-f16 ceiling (dense f16 MFMA / 3 products)"},
                         "whole_forward": {"compulsory_bytes_per_seq": model_compulsory_bytes(opts),
                                           "achieved_gbs": round(whole_bytes, 1),
                                           "frac_hbm": round(whole_bytes / PEAK_HBM_GBS, 4),
                                           "flop_per_seq": total_flop_per_seq,
                                           "achieved_tflops": round(total_flop_per_seq * G * args.steps / elapsed / 1e12,
                                                                    3)}},
            "kernel_ms_per_step_event_bracketed": {native.KIND_NAMES[k]: round(v / args.steps, 4)
                                                   for k, v in sorted(per_kind.items())},
            "host_us_per_call": round(host_s / args.steps * 1e6, 2),
            "timed_call": "model(x): DSTDGCN.forward (the drop-in path) -> eager: DSTDGCN._forward_native -> "
                          "dstd_model_fwd_ex, the implementation of torch.ops.dstd.dstdgcn_forward without the "
                          "dispatcher's boxing (the op itself runs under tracing / torch.compile)",
        }
        side_cpu = None if args.no_cpu_baseline else args.side_cpu_seconds
        if world == 1 and args.config == "h36m" and not args.no_variant:
            out["variant_t75"] = config_leg("h36m75", B, device, args.steps, args.warmup, side_cpu)
            out["cmu_b256"] = config_leg("cmu", B, device, args.steps, args.warmup, side_cpu)
            out["3dpw_b256"] = config_leg("3dpw", B, device, args.steps, args.warmup, side_cpu)
        if world == 1 and not args.no_side:
            out["exact_fp32"] = arithmetic_leg(model, x, "fp32", args.steps, args.warmup)
            out["eval_b32"] = small_batch_leg(model, x, 32, max(args.steps, 100), args.warmup)
            out["train_b32"] = train_leg(device, 32, 20, 5)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(opts, sd, x_cpu, args.cpu_seconds, 30.0)
            out["vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
