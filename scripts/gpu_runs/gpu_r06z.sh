#!/bin/bash
# round 6 (r06z): which part of a live RCCL process group slows the forward
# ~4% (r06y: gloo under torchrun does not): torch's NCCL watchdog / monitor
# threads off, RCCL's cuMem and MSCCL paths off
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06z
mkdir -p $O
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u $B > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 300 $TR --master-port 29551 $B > $O/nccl.json 2> $O/nccl.err || exit 1
TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_DUMP_ON_TIMEOUT=0 \
  timeout -k 10 300 $TR --master-port 29552 $B > $O/nccl_nomon.json 2> $O/nccl_nomon.err || exit 1
NCCL_CUMEM_ENABLE=0 timeout -k 10 300 $TR --master-port 29553 $B > $O/nccl_nocumem.json 2> $O/nccl_nocumem.err || exit 1
RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 timeout -k 10 300 $TR --master-port 29554 $B > $O/nccl_nomsccl.json 2> $O/nccl_nomsccl.err || exit 1
python3 - <<'PY'
import json
for n in ("plain", "nccl", "nccl_nomon", "nccl_nocumem", "nccl_nomsccl"):
    d = json.loads(open(f"gpurun_out/r06z/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["host_us_per_call"], d["roofline"]["avg_launch_us"])
PY
