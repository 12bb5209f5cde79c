#!/bin/bash
# round 5 (r05aa): after the 8-wave spatial aggregation backward (default):
# BN row batches of 16 instead of 8 (rb16: the statistics pass holds a
# config-5 chunk in registers), frame-split targets 3 / 1 for the
# aggregation backward (b3 / b1): training suite, B=32 step A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2 3; do
  for v in new rb16 b3 b1; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05aa/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"])
PY
