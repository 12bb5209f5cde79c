#!/bin/bash
# round 4 (r04ag): streaming GEMM addressing -- one lane base per operand, rows
# past K / M left to the buffer range (HEAD) vs per-load bounds (prev) -- training
# suites on HEAD, then the B=32 / B=256 step A/B
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; echo "suites: $(tail -1 $O/pytest_train.log)"; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_prev libdstd_gcn; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
  done
done
timeout -k 10 60 scripts/micro/skinny_micro > $O/micro.txt 2>&1; st=$?; cat $O/micro.txt; [ $st -eq 0 ] || exit $st
