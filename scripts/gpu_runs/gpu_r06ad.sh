#!/bin/bash
# round 6 (r06ad): final tree -- the whole GPU suite, smoke(), the driver's
# bench command, and the rocprofv3 kernel-trace + FETCH/WRITE PMC passes
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ad
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
st=$?; tail -2 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
st=$?; tail -1 $O/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
st=$?; tail -c 300 $O/bench.json; [ $st -eq 0 ] || exit $st
PROF_TAG=r06ad bash scripts/gpu_profile.sh
