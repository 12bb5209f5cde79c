#!/bin/bash
# round 5 (r05z): the spatial aggregation backward (k_aggc_bwd<false, JF>) with
# 8 waves per workgroup instead of 4 (t512; t512b0 / t512b4: frame-split
# target 0 / 4 instead of 2): training suite on t512 (DSTD_LIB), then the B=32
# step A/B (3 interleaved rounds)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05z
mkdir -p $O
DSTD_LIB=$R/dstd-gcn_amd/libdstd_gcn_t512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2 3; do
  for v in new t512 t512b0 t512b4; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05z/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"])
PY
