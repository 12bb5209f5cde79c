#!/bin/bash
# round 6 (r06o): static VALU priority for the younger waves during the block
# kernel's spatial units (DSTD_BF_SETPRIO 1 / 2 / 3) against none -- parity
# suite, then A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06o
mkdir -p $O
L=$R/dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "block_fused or large_batch" > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_prio1.so $L/libdstd_gcn_prio2.so $L/libdstd_gcn_prio3.so \
    --config $cfg --rounds 7 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; grep wall $O/ab_$cfg.txt | tail -4
done
