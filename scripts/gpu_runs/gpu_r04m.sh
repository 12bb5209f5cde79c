#!/bin/bash
# round 4 (r04m): forward parity suite; same-box A/B of HEAD against the
# previous commit (prev): the encoder residual as the aggregation
# accumulator's initial value at T = 40 (3DPW; its fused kernel's spills gone)
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04m
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in 3dpw h36m; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config $cfg --rounds 7 >> $O/ab.txt 2>&1 || exit 1
done
echo "# 3dpw B=32" >> $O/ab.txt
timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config 3dpw --batch 32 --rounds 5 --steps 20 >> $O/ab.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
