#!/bin/bash
# round 6 (r06x): order check for r06w's plain vs torchrun N=1 gap at B=256 --
# alternating, torchrun first
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06x
mkdir -p $O
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 2953$i $B > $O/dist1_$i.json 2> $O/dist1_$i.err || exit 1
  timeout -k 10 300 python -u $B > $O/plain_$i.json 2> $O/plain_$i.err || exit 1
done
python3 - <<'PY'
import json
for n in ("dist1_1", "plain_1", "dist1_2", "plain_2"):
    d = json.loads(open(f"gpurun_out/r06x/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["host_us_per_call"], d["roofline"]["avg_launch_us"])
PY
