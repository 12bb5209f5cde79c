#!/bin/bash
# round 5 (r05g): (4x bar, 10 noise samples) the measured fp32 noise floor in every whole-model step test,
# the per-block bisection test, grad_tail_bisect.py tables
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r05g
mkdir -p $O
true

timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_dp8.py -k "model_step or syncbn or config5 or tail" > $O/pytest.log 2>&1
st=$?; grep -E "noise floor|PASS|FAIL|Error|assert" $O/pytest.log | head -40; exit $st
