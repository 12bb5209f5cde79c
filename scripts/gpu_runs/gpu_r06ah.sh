#!/bin/bash
# round 6 (r06ah): the whole GPU suite and smoke() on the final tree
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ah
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
st=$?; tail -2 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
st=$?; tail -1 $O/smoke.log; exit $st
