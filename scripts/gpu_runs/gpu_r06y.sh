#!/bin/bash
# round 6 (r06y): where the torchrun N=1 bench loses 3.5-4.9% at B=256
# (r06w/x): torchrun + gloo, torchrun + lazily initialised RCCL, plain with
# torchrun's OMP_NUM_THREADS=1, against plain and torchrun + RCCL (default)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06y
mkdir -p $O
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u $B > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 300 $TR --master-port 29541 $B > $O/dist_nccl.json 2> $O/dist_nccl.err || exit 1
DSTD_BENCH_BACKEND=gloo timeout -k 10 300 $TR --master-port 29542 $B > $O/dist_gloo.json 2> $O/dist_gloo.err || exit 1
DSTD_BENCH_EAGER_INIT=0 timeout -k 10 300 $TR --master-port 29543 $B > $O/dist_lazy.json 2> $O/dist_lazy.err || exit 1
OMP_NUM_THREADS=1 timeout -k 10 300 python -u $B > $O/plain_omp1.json 2> $O/plain_omp1.err || exit 1
timeout -k 10 300 python -u $B > $O/plain2.json 2> $O/plain2.err || exit 1
python3 - <<'PY'
import json
for n in ("plain", "dist_nccl", "dist_gloo", "dist_lazy", "plain_omp1", "plain2"):
    d = json.loads(open(f"gpurun_out/r06y/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["host_us_per_call"], d["roofline"]["avg_launch_us"])
PY
