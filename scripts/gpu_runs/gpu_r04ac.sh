#!/bin/bash
# round 4 (r04ac): final HEAD -- whole GPU suite, smoke, the B=32 / B=256
# training step
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; echo "suite: $(tail -1 $O/pytest_gpu.log)"; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; grep -v amdgpu.ids $O/smoke.log | tail -2; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train.log 2>&1
st=$?; grep metric $O/train.log | cut -c1-110; [ $st -eq 0 ] || exit $st
