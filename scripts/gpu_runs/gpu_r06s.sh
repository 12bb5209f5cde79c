#!/bin/bash
# round 6 (r06s): the driver's bench command on the final forward tree, then the
# rocprofv3 kernel-trace/stats pass and the FETCH_SIZE / WRITE_SIZE PMC passes
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
st=$?; tail -c 400 $O/bench.json; [ $st -eq 0 ] || exit $st
PROF_TAG=r06s bash scripts/gpu_profile.sh
