#!/bin/bash
# round 4 (r04r): streaming 1x1-conv GEMM diagnostics -- microbenchmark of the
# default build against the panel / tile kernels (nostream), fewer resident
# workgroups (csg2 / csg4: more items per wave), no MFMAs (csnomfma), no
# stores (csnost), 32 / 64-column items (nt2, nt2n, nt4n: n = no prefetch); then the training suites with HEAD (shared-A routing fix)
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04r
mkdir -p $O
for v in nostream "" csg2 csg4 csnomfma csnost nt2 nt2n nt4n; do
  b=scripts/micro/skinny_micro${v:+_$v}
  timeout -k 10 60 $b > $O/micro_${v:-stream}.txt 2>&1; st=$?
  echo "== ${v:-stream} (exit $st)"; cat $O/micro_${v:-stream}.txt | grep -v FAIL | tail -1
  [ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -2 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
# training step A/B at B=32: panel / tile GEMMs (nostream) vs HEAD (streaming
# GEMM), and HEAD with 4 samples per BN-apply workgroup (bnns4, bnns4eb8) or
# the BN merges as launches of their own + flat float4 applies, both
# directions (bnsep)
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_nostream libdstd_gcn libdstd_gcn_bnns4 libdstd_gcn_bnns4eb8 libdstd_gcn_bnsep; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 200 python -u scripts/bench_train.py --batch 32 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st $(grep metric $O/train_$lib.$r.log | cut -c1-110)"; [ $st -eq 0 ] || exit $st
  done
done
# the bnsep variant against the block / model-step parity tests
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_bnsep.so" timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py -k "dstdgcb or model_step or forward_pair" > $O/pytest_bnsep.log 2>&1
st=$?; echo "bnsep parity: $(tail -1 $O/pytest_bnsep.log)"; [ $st -eq 0 ] || exit $st
