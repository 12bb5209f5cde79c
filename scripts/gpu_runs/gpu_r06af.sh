#!/bin/bash
# round 6 (r06af): the first bench process on a fresh box with the untimed
# settle period (default 300 ms) -- K=20 first, then settle off, then K=200
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06af
mkdir -p $O
A="--gpus 1 --no-variant --no-side --no-cpu-baseline --warmup 5"
timeout -k 10 300 python -u bench.py $A --steps 20 > $O/first_settle.json 2> $O/first_settle.err || exit 1
timeout -k 10 300 python -u bench.py $A --steps 20 --settle-ms 0 > $O/nosettle.json 2> $O/nosettle.err || exit 1
timeout -k 10 300 python -u bench.py $A --steps 20 > $O/settle2.json 2> $O/settle2.err || exit 1
timeout -k 10 300 python -u bench.py $A --steps 200 > $O/s200.json 2> $O/s200.err || exit 1
python3 - <<'PY'
import json
for n in ("first_settle", "nosettle", "settle2", "s200"):
    d = json.loads(open(f"gpurun_out/r06af/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["settle"]["steps"], d["roofline"]["avg_launch_us"])
PY
