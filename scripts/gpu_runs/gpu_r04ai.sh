#!/bin/bash
# round 4 (r04ai): the streaming GEMM's item width again after the addressing
# change (nt2: 32-column items with the next-item prefetch, nt2n: without)
# -- the nt2 variant on the training suites, then the B=32 / B=256 step A/B
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04ai
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_nt2.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_nt2.log 2>&1
st=$?; echo "nt2 suites: $(tail -1 $O/pytest_nt2.log)"; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_nt2 libdstd_gcn_nt2n; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-100; [ $st -eq 0 ] || exit $st
  done
done
