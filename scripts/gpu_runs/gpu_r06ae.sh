#!/bin/bash
# round 6 (r06ae): does the driver's short run (20 timed steps after 5
# warm-up + the untimed profiled pass) read slower than a long one?
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ae
mkdir -p $O
A="--gpus 1 --no-variant --no-side --no-cpu-baseline"
for s in 20 20 200; do
  timeout -k 10 300 python -u bench.py $A --steps $s --warmup 5 > $O/s$s.json 2> $O/s$s.err || exit 1
  python3 -c "
import json
d = json.loads(open('$O/s$s.json').read().strip().splitlines()[-1])
print('steps $s', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
