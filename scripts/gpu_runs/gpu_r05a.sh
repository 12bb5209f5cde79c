#!/bin/bash
# round 5 (r05a): configs 4 / 5 at their shapes (world-8 gloo on the one GPU),
# the data-parallel suite and the backward error-path join
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_dp8.py -s > $O/pytest_dp.log 2>&1
st=$?; grep -E "PASS|FAIL|ERROR|median|picks|passed|failed" $O/pytest_dp.log | tail -30; exit $st
