#!/bin/bash
# round 5 (r05m): anchored parameter inputs of the training Function in the
# in-place gradient mode (host time of the step), training / engine / dist /
# dp8 suites; B=32 graph replay by input-copy kind
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py tests/test_gpu_dist.py tests/test_gpu_dp8.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2 3; do
  timeout -k 10 200 python -u scripts/train_host_split.py 2>&1 | grep -v amdgpu.ids >> $O/host_split.txt || exit 1
done
cat $O/host_split.txt
for r in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 new 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05m/train_b32.txt"):
    if " {" in l:
        d = json.loads(l.split(" ", 1)[1])
        print("B=32 ms", d["ms_per_step"], "host_us", d["host_us_per_step"], "host_issue_us", d["host_issue_us_per_step"], "graph ms", d["graph_replay"]["ms_per_step"])
PY
timeout -k 10 200 python -u scripts/graph_copy_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/graph_copy.txt
