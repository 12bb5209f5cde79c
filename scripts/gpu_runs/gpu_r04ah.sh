#!/bin/bash
# round 4 (r04ah): final HEAD -- whole GPU suite, smoke, the full bench line
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04ah
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; echo "suite: $(tail -1 $O/pytest_gpu.log)"; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; grep -v amdgpu.ids $O/smoke.log | tail -2; [ $st -eq 0 ] || exit $st
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 300 $O/bench.json; [ $st -eq 0 ] || exit $st
