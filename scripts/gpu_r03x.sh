#!/bin/bash
# round 3 (r03x): GPU suite + smoke + full bench line at HEAD (fused Adam in
# the engine / train leg), kernel trace of the training step
cd "$(dirname "$0")/.." || exit 2
R="$PWD"
O=$R/gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; tail -3 $O/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 2500 $O/bench.json; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/scripts/train_prof.py" 32 10 > "$O/kt.log" 2>&1)
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/kt/run_kernel_trace.csv 10 60 > $O/train_trace_summary.txt; head -12 $O/train_trace_summary.txt
