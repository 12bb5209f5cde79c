#!/bin/bash
# round 3 (r03w, re-entry): GPU suite + smoke, training A/B of the fused
# dM + tanh backward (default) against the dM GEMM + tanh pair
# (DSTD_TRAIN_DM_GEMM=1), training host-time probe per phase, kernel trace of
# the training step, full bench line
cd "$(dirname "$0")/.." || exit 2
R="$PWD"
O=$R/gpurun_out/r03w
mkdir -p $O
DSTD_TRAIN_TANH_FUSED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for i in 1 2; do
  DSTD_TRAIN_TANH_FUSED=1 timeout -k 10 200 python -u scripts/train_ab.py 32 fused >> $O/ab.txt 2>&1 || exit 1
  timeout -k 10 200 python -u scripts/train_ab.py 32 default >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-10,130-300
DSTD_TRAIN_TANH_FUSED=1 timeout -k 10 200 python -u scripts/train_host_probe.py > $O/host_probe.txt 2>&1; st=$?; grep -v amdgpu.ids $O/host_probe.txt; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(export DSTD_TRAIN_TANH_FUSED=1; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/scripts/train_prof.py" 32 10 > "$O/kt.log" 2>&1)
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/kt/run_kernel_trace.csv 10 60 > $O/train_trace_summary.txt; head -45 $O/train_trace_summary.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; tail -3 $O/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 1500 $O/bench.json; exit $st
