#!/bin/bash
# round 4 (r04l): training suite; B=32 / B=256 training step A/B of HEAD
# against the previous commit (prev): the strided GEMM's adjacency epilogue
# (conv_rm -> E and D = alpha E + A_comb) loads the combine once per column
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04l
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_prev libdstd_gcn; do
    DSTD_LIB="$R/$L/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-200; [ $st -eq 0 ] || exit $st
  done
done
