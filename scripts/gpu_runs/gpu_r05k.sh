#!/bin/bash
# round 5 (r05k): host side of the training step -- forward_pair's two-output
# Function and the engine's LeanAdam: training / engine / dp suites, host
# split of the step (LeanAdam vs torch Adam), bench train leg
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05k
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py tests/test_gpu_dist.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  timeout -k 10 200 python -u scripts/train_host_split.py 2>&1 | grep -v amdgpu.ids | sed 's/^/lean /' >> $O/host_split.txt || exit 1
  TORCH_ADAM=1 timeout -k 10 200 python -u scripts/train_host_split.py 2>&1 | grep -v amdgpu.ids | sed 's/^/torch /' >> $O/host_split.txt || exit 1
done
cat $O/host_split.txt
for r in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 new 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05k/train_b32.txt"):
    if " {" in l:
        d = json.loads(l.split(" ", 1)[1])
        print("B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"], "graph ms", d["graph_replay"]["ms_per_step"])
PY
