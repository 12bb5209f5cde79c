#!/bin/bash
# round 6 (r06f): the gradient-bar calibration with the fp64 PReLU-slope
# partials, then the whole GPU suite without -x (every test that misses the
# calibrated 3x bar, not just the first)
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u scripts/grad_bar_calibration.py $O/grad_bar_calibration.json > $O/grad_bar.txt 2>&1 || exit 1
tail -4 $O/grad_bar.txt
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
st=$?; grep -E "FAILED|passed|failed" $O/pytest_gpu.log | tail -8; grep "noise floor" $O/pytest_gpu.log | head -20; exit $st
