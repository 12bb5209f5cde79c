#!/bin/bash
# A/B of training-step library variants on one box: for each library in
# AB_LIBS, the training parity tests then the B=32/256 training bench.
REPO="$(cd "$(dirname "$0")/.." && pwd)"
cd "$REPO" || exit 2
mkdir -p gpurun_out/ab
for lib in ${AB_LIBS:-dstd-gcn_amd/libdstd_gcn.so}; do
  tag=$(basename "$lib" .so)
  DSTD_LIB="$REPO/$lib" timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/$tag.tests.log 2>&1
  st=$?; echo "$tag tests exit $st"; tail -2 gpurun_out/ab/$tag.tests.log; [ $st -le 1 ] || exit $st
done
for r in 1 2; do
  for lib in ${AB_LIBS:-dstd-gcn_amd/libdstd_gcn.so}; do
    tag=$(basename "$lib" .so)
    DSTD_LIB="$REPO/$lib" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > gpurun_out/ab/$tag.bench$r.log 2>&1
    st=$?; echo "$tag bench$r exit $st"; grep metric gpurun_out/ab/$tag.bench$r.log | cut -c1-300; [ $st -eq 0 ] || exit $st
  done
done
