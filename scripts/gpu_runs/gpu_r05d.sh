#!/bin/bash
# round 5 (r05d): d alpha in fp64 partials -- grad_tail_bisect.py again, then
# the training suite
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u scripts/grad_tail_bisect.py > $O/grad_tail.txt 2>&1
st=$?; grep -v amdgpu.ids $O/grad_tail.txt | head -30; [ $st -eq 0 ] || exit $st
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_dist.py > $O/pytest_train.log 2>&1
st=$?; tail -3 $O/pytest_train.log; exit $st
