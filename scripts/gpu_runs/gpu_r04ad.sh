#!/bin/bash
# round 4 (r04ad): samples per BN-apply workgroup at the config-5 batch
# (HEAD: 1 at B=32; bnns2 / bnns4: 2 / 4 -- half / a quarter of the per-
# workgroup merges), training step A/B, parity of bnns4 on the training suite
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04ad
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_bnns4.so" timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py > $O/pytest_bnns4.log 2>&1
st=$?; echo "bnns4 suite: $(tail -1 $O/pytest_bnns4.log)"; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_bnns2 libdstd_gcn_bnns4; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 200 python -u scripts/bench_train.py --batch 32 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st $(grep metric $O/train_$lib.$r.log | cut -c1-100)"; [ $st -eq 0 ] || exit $st
  done
done
