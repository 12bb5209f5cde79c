#!/bin/bash
# round 4 (r04q): the streaming 1x1-conv GEMM (k_conv_stream) -- microbenchmark
# and host-reference check against the panel / tile kernels (nostream build),
# the GEMM shape log of one B=32 training step, the training suites, then the
# B=32 / B=256 training step A/B nostream vs HEAD
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04q
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 60 scripts/micro/skinny_micro_nostream > $O/micro_nostream.txt 2>&1; st=$?; cat $O/micro_nostream.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 60 scripts/micro/skinny_micro > $O/micro_stream.txt 2>&1; st=$?; cat $O/micro_stream.txt; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
DSTD_LIB="$R/$L/libdstd_gcn_gemmlog.so" timeout -k 10 200 python -u scripts/bench_train.py --batch 32 --steps 2 --warmup 1 > $O/gemmlog.out 2> $O/gemmlog.txt
st=$?; echo "gemmlog exit $st, $(grep -c '^gemm' $O/gemmlog.txt) lines"; [ $st -eq 0 ] || exit $st
unset DSTD_AB_FOREIGN_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_nostream libdstd_gcn; do
    DSTD_LIB="$R/$L/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-130; [ $st -eq 0 ] || exit $st
  done
done
