#!/bin/bash
# round 6 (r06p): younger-wave priority in the spatial units now default (main);
# against it off (prio0) and the same in phase 2 (tp2), phase 3 (tp3), both
# (tp23) -- parity subset, then A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06p
mkdir -p $O
L=$R/dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "block_fused or large_batch" > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_prio0.so $L/libdstd_gcn_tp2.so $L/libdstd_gcn_tp3.so $L/libdstd_gcn_tp23.so \
    --config $cfg --rounds 7 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; grep wall $O/ab_$cfg.txt | tail -5
done
