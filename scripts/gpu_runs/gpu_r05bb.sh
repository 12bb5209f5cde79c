#!/bin/bash
# round 5 (r05bb): an op's three weight-gradient finishes (adjacency finish,
# dW_rm and [dWp | db] split-K finishes) as one launch on the second stream
# (finish_set; sepfin = three launches as before): graphed / stream tests,
# training suites, B=32 (3 rounds) / B=256 A/B, launches per step
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05bb
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "graphed or wgrad_stream" > $O/pytest_graphed.log 2>&1
st=$?; tail -1 $O/pytest_graphed.log; [ $st -eq 0 ] || exit $st
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py tests/test_gpu_dist.py tests/test_gpu_dp8.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2 3; do
  for v in sepfin new; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
for v in sepfin new; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 300 python -u scripts/bench_train.py --batch 256 --steps 10 --warmup 3 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/train_b256.txt || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05bb/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"])
PY
cat $O/train_b256.txt

timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tt -o run -- python3 scripts/bench_train.py --batch 32 --steps 6 --warmup 3 > $O/tt.log 2>&1 || exit 1
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt || exit 1
head -3 $O/train_trace_summary.txt; tail -2 $O/train_trace_summary.txt
