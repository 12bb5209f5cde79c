#!/bin/bash
# round 5 (r05hh): spatial backward aggregation at 64 channels per workgroup
# as the default (cw16 = the 16-channel chunks before; cw64s1 = 64 channels
# with one workgroup per CU aimed at instead of two: 8 frames per workgroup):
# training GPU suites on the new default, gradients compared, B=32 A/B (3
# rounds), B=256 step
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05hh
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py tests/test_gpu_dist.py tests/test_gpu_dp8.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for v in new cw16 cw64s1; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/grad_ab.py $O/g_$v.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python3 scripts/grad_ab.py --compare $O/g_cw16.npz $O/g_new.npz && python3 scripts/grad_ab.py --compare $O/g_new.npz $O/g_cw64s1.npz || exit 1
for r in 1 2 3; do
  for v in new cw16 cw64s1; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05hh/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"])
PY
for v in new cw16; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 300 python -u scripts/bench_train.py --batch 256 --steps 10 --warmup 3 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/train_b256.txt || exit 1
done
cat $O/train_b256.txt
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tt -o run -- python3 scripts/bench_train.py --batch 32 --steps 6 --warmup 3 > $O/tt.log 2>&1 || exit 1
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt || exit 1
head -2 $O/train_trace_summary.txt | tail -1; grep -E "k_aggc_bwd|k_adj_bwd_part" $O/train_trace_summary.txt; tail -2 $O/train_trace_summary.txt
