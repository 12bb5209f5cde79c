#!/bin/bash
# round 6 (r06al): bench.py's N>1 path rehearsed with 2 and 4 ranks sharing the
# box's one GPU over gloo (scripts/bench_shared_gpu.py): broadcast, barriers,
# settle, timed region, MAX / checksum exchange, the rank-0 JSON line
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06al
mkdir -p $O
A="--no-variant --no-side --no-cpu-baseline --steps 20 --warmup 5"
for n in 2 4; do
  DSTD_BENCH_BACKEND=gloo timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2958$n scripts/bench_shared_gpu.py --gpus $n $A > $O/n$n.json 2> $O/n$n.err || exit 1
  python3 -c "
import json
d = json.loads(open('$O/n$n.json').read().strip().splitlines()[-1])
print('n=$n', d['n_gpus'], d['value'], d['ms_per_step'], d['scaling'], d['config']['global_batch'], d['config']['parallelism'])"
done
