#!/bin/bash
# round 5 (r05jj): the train-mode spatial forward aggregation (k_aggc) over
# 64 channels per workgroup (fcw64) vs 16-channel chunks (default); the
# backward's row-tile count fixed for 33..48 channels (3 runs as 4): op and
# block training tests on both builds, gradients compared, B=32 A/B (3
# rounds), B=256 step
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05jj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "op_backward or red_channels or dstdgcb_train" > $O/pytest_ops.log 2>&1
st=$?; tail -1 $O/pytest_ops.log; [ $st -eq 0 ] || exit $st
DSTD_LIB=$R/dstd-gcn_amd/libdstd_gcn_fcw64.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "op_backward or red_channels or dstdgcb_train" > $O/pytest_ops_fcw64.log 2>&1
st=$?; tail -1 $O/pytest_ops_fcw64.log; [ $st -eq 0 ] || exit $st
for v in new fcw64; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/grad_ab.py $O/g_$v.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python3 scripts/grad_ab.py --compare $O/g_new.npz $O/g_fcw64.npz || exit 1
for r in 1 2 3; do
  for v in new fcw64; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05jj/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"])
PY
for v in new fcw64; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 300 python -u scripts/bench_train.py --batch 256 --steps 10 --warmup 3 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/train_b256.txt || exit 1
done
cut -c1-120 $O/train_b256.txt
