#!/bin/bash
# round 6 (r06ac): is the RCCL-alive slowdown ROCm SMI initialisation?  plain
# bench, bench after rsmi_init / amdsmi_init in the process, torchrun + RCCL
# bound at init (the slow case)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ac
mkdir -p $O
A="--gpus 1 --no-variant --no-side --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 300 python -u scripts/rsmi_probe.py rsmi $A > $O/rsmi.json 2> $O/rsmi.err || exit 1
timeout -k 10 300 python -u scripts/rsmi_probe.py amdsmi $A > $O/amdsmi.json 2> $O/amdsmi.err || exit 1
DSTD_BENCH_RCCL_EARLY=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py $A > $O/rccl_early.json 2> $O/rccl_early.err || exit 1
timeout -k 10 300 python -u bench.py $A > $O/plain2.json 2> $O/plain2.err || exit 1
grep -h "init" $O/rsmi.err $O/amdsmi.err
python3 - <<'PY'
import json
for n in ("plain", "rsmi", "amdsmi", "rccl_early", "plain2"):
    d = json.loads(open(f"gpurun_out/r06ac/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])
PY
