#!/bin/bash
# round 5 (r05q): the frame split of the channel-chunk aggregation kernels
# per direction: f<k>b<k> = forward / backward split target in workgroups per
# CU (0 = none; default f2b2): B=32 training step A/B (2 interleaved rounds);
# training suite on the default
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for v in f0b0 f2b0 f0b2 new f4b0; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05q/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"])
PY
