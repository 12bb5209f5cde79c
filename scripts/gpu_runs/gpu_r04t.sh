#!/bin/bash
# round 4 (r04t): validation first, then measurement.
#  1. training + channels-last suites on HEAD (streaming GEMM for the
#     shared-weight products, adjacency-backward partials over column blocks)
#  2. streaming-GEMM microbenchmark: panel / tile kernels (nostream), default,
#     no MFMAs (csnomfma), no stores (csnost), 32-column items without
#     prefetch (nt2n), half the resident workgroups (csg2)
#  3. training step A/B, B=32 / 256: prev (HEAD before the adjacency change),
#     nostream and bnsep (prev + that one switch), HEAD
#  4. the bnsep variant against the block / model-step parity tests
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for v in nostream "" csnomfma csnost nt2n csg2; do
  b=scripts/micro/skinny_micro${v:+_$v}
  timeout -k 10 60 $b > $O/micro_${v:-stream}.txt 2>&1; st=$?
  echo "== ${v:-stream} (exit $st): $(tail -1 $O/micro_${v:-stream}.txt)"
  [ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
done
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_prev libdstd_gcn_nostream libdstd_gcn_bnsep libdstd_gcn; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
  done
done
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_bnsep.so" timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py -k "dstdgcb or model_step or forward_pair" > $O/pytest_bnsep.log 2>&1
st=$?; echo "bnsep parity: $(tail -1 $O/pytest_bnsep.log)"; [ $st -eq 0 ] || exit $st
