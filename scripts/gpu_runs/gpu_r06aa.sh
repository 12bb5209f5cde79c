#!/bin/bash
# round 6 (r06aa): bench with RCCL kept out of the timed region (gloo group for
# the weight broadcast and the barriers, RCCL for the MAX / checksum after it)
# -- torchrun N=1 against plain N=1 and against RCCL bound at init (as before)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06aa
mkdir -p $O
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u $B > $O/plain_b256.json 2> $O/plain_b256.err || exit 1
timeout -k 10 300 $TR --master-port 29561 $B > $O/dist1_b256.json 2> $O/dist1_b256.err || exit 1
DSTD_BENCH_RCCL_EARLY=1 timeout -k 10 300 $TR --master-port 29562 $B > $O/dist1_early_b256.json 2> $O/dist1_early_b256.err || exit 1
timeout -k 10 300 python -u $B --global-batch 2048 > $O/plain_g2048.json 2> $O/plain_g2048.err || exit 1
timeout -k 10 300 $TR --master-port 29563 $B --global-batch 2048 > $O/dist1_g2048.json 2> $O/dist1_g2048.err || exit 1
timeout -k 10 300 $TR --master-port 29564 $B > $O/dist1_b256_2.json 2> $O/dist1_b256_2.err || exit 1
python3 - <<'PY'
import json
for n in ("plain_b256", "dist1_b256", "dist1_early_b256", "plain_g2048", "dist1_g2048", "dist1_b256_2"):
    d = json.loads(open(f"gpurun_out/r06aa/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["n_gpus"], d["scaling"], d["config"]["global_batch"],
          d["roofline"]["avg_launch_us"])
PY
