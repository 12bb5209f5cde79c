#!/bin/bash
# round 4 (r04z): the separate BN merge now chosen by size (>= 2^24 elements:
# the B=256 step) -- whole GPU suite on HEAD, then the B=32 / B=256 step
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; echo "suite: $(tail -1 $O/pytest_gpu.log)"; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train.$r.log 2>&1
  st=$?; echo "round $r exit $st"; grep metric $O/train.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
done
