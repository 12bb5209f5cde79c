#!/bin/bash
# round 5 (r05ll): final state of the round (after the row-tile fix of r05jj) --
# whole GPU suite, smoke, the bench line and the B=32 training trace
# training step's kernel trace (forward kernels unchanged since r05cc: its
# forward traces and HBM passes stand)
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r05ll
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -2 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; grep -v amdgpu.ids $O/smoke.log | tail -3; [ $st -eq 0 ] || exit $st
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 600 $O/bench.json; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tt" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 6 --warmup 3 > "$O/tt.log" 2>&1)
st=$?; echo "train trace exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt
head -2 $O/train_trace_summary.txt; tail -2 $O/train_trace_summary.txt
