#!/bin/bash
# round 6 (r06k): bisect r06j's sample-independence failure over the phase-3
# TPI and the phase-2 stage split (main = split + TPI 2, sp1 = split + TPI 1,
# p3t2 / p3t1 = no split)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06k
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for v in "" _sp1 _p3t2 _p3t1; do
  DSTD_LIB=$L/libdstd_gcn$v.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "large_batch or block_fused_schedule or fused_temporal_schedule" > $O/pytest$v.log 2>&1
  st=$?; echo "lib$v rc=$st: $(tail -1 $O/pytest$v.log)"
  [ $st -le 1 ] || exit $st
done
