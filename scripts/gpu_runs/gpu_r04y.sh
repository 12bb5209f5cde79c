#!/bin/bash
# round 4 (r04y): DSTD_BN_SEP again with 32-bit indexing in its flat applies
# (r04u measured it with 64-bit divides per float4: B=32 +6%) -- parity of the
# variant on the block / model-step / forward-pair tests, then the training
# step A/B against HEAD
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04y
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
DSTD_LIB="$R/dstd-gcn_amd/libdstd_gcn_bnsep.so" timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_bnsep.log 2>&1
st=$?; echo "bnsep suites: $(tail -1 $O/pytest_bnsep.log)"; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_bnsep; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
  done
done
