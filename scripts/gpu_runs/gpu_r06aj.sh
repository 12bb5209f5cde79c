#!/bin/bash
# round 6 (r06aj): the driver's bench command after the last bench.py edits
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06aj
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
st=$?; tail -c 600 $O/bench.json; exit $st
