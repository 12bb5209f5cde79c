#!/bin/bash
# round 3 (r03y): 96-wide tiles for the reduce GEMMs (packed-conv [W | b] and
# conv_rm weight gradients; opt-in DSTD_GEMM_96=1) -- training tests, same-box
# A/B against the 64-wide tiles, GPU suite + smoke + bench line, training kernel trace
cd "$(dirname "$0")/.." || exit 2
R="$PWD"
O=$R/gpurun_out/r03y
mkdir -p $O
DSTD_GEMM_96=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for i in 1 2; do
  DSTD_GEMM_96=1 timeout -k 10 200 python -u scripts/train_ab.py 32 t96 >> $O/ab.txt 2>&1 || exit 1
  timeout -k 10 200 python -u scripts/train_ab.py 32 t64 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-10,130-300
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; tail -3 $O/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 800 $O/bench.json; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(export DSTD_GEMM_96=1; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/scripts/train_prof.py" 32 10 > "$O/kt.log" 2>&1)
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/kt/run_kernel_trace.csv 10 60 > $O/train_trace_summary.txt; head -12 $O/train_trace_summary.txt
