#!/bin/bash
# round 6 (r06w): the bench's RCCL path at one rank on the final tree
# (VERDICT r05 item 6): plain N=1 and torchrun N=1 at B=256 and at config 4's
# global batch 2048 on one GPU
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06w
mkdir -p $O
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
timeout -k 10 300 python -u $B > $O/plain_b256.json 2> $O/plain_b256.err || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 $B > $O/dist1_b256.json 2> $O/dist1_b256.err || exit 1
timeout -k 10 300 python -u $B --global-batch 2048 > $O/plain_g2048.json 2> $O/plain_g2048.err || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29532 $B --global-batch 2048 > $O/dist1_g2048.json 2> $O/dist1_g2048.err || exit 1
python3 - <<'PY'
import json
for n in ("plain_b256", "dist1_b256", "plain_g2048", "dist1_g2048"):
    d = json.loads(open(f"gpurun_out/r06w/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["scaling"], d["config"]["global_batch"], d["roofline"]["kernel"],
          d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
PY
