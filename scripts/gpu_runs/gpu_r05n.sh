#!/bin/bash
# round 5 (r05n): anchored parameter inputs of the training Function
# (in-place gradient mode) and the frame-split channel-chunk aggregation
# kernels (k_aggc / k_aggc_bwd, spatial): training / dist / dp8 / parity
# suites, host split, B=32 step A/B by split target (0 = none, 2, 4 default, 8
# workgroups per CU), B=32 graph replay by input-copy kind
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05n
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py tests/test_gpu_dist.py tests/test_gpu_dp8.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2 3; do
  timeout -k 10 200 python -u scripts/train_host_split.py 2>&1 | grep -v amdgpu.ids >> $O/host_split.txt || exit 1
done
cat $O/host_split.txt
for r in 1 2; do
  for v in agg0 agg2 new agg8; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib DSTD_AB_FOREIGN_LIB=1 timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05n/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_us", d["host_us_per_step"], "host_issue_us", d["host_issue_us_per_step"], "graph ms", d["graph_replay"]["ms_per_step"])
PY
timeout -k 10 200 python -u scripts/graph_copy_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/graph_copy.txt
