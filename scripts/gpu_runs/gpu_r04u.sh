#!/bin/bash
# round 4 (r04u): the three training switches, off by default, validated and
# measured before any is turned on:
#   stream   -DDSTD_GEMM_STREAM=1 (shared-weight products on k_conv_stream)
#   adjsplit -DDSTD_ADJ_SPLIT     (adjacency-backward partials over column blocks)
#   bnsep    -DDSTD_BN_SEP        (BN merges as launches of their own, flat applies)
#   all3     all of them
#  1. training + channels-last suites on all3 (DSTD_LIB), then on HEAD
#  2. microbenchmark: panel / tile kernels (HEAD), stream, and stream with no
#     MFMAs / no stores / 32-column items / half the workgroups
#  3. training step A/B, B=32 / 256, two rounds: HEAD, stream, adjsplit, bnsep, all3
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04u
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_all3.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_all3.log 2>&1
st=$?; echo "all3 suites: $(tail -1 $O/pytest_all3.log)"; [ $st -eq 0 ] || exit $st
unset DSTD_AB_FOREIGN_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_head.log 2>&1
st=$?; echo "HEAD suites: $(tail -1 $O/pytest_head.log)"; [ $st -eq 0 ] || exit $st
for v in "" stream csnomfma csnost nt2n csg2; do
  b=scripts/micro/skinny_micro${v:+_$v}
  timeout -k 10 60 $b > $O/micro_${v:-head}.txt 2>&1; st=$?
  echo "== ${v:-head} (exit $st): $(tail -1 $O/micro_${v:-head}.txt)"
  [ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
done
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_stream libdstd_gcn_adjsplit libdstd_gcn_bnsep libdstd_gcn_all3; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
  done
done
