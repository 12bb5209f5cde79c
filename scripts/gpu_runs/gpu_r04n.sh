#!/bin/bash
# round 4 (r04n): same-box A/B of HEAD against ra35 (the encoder residual as
# the accumulator's initial value at T = 35 too: 48 VALU adds per unit fewer,
# but 3 VGPRs spilled in the 12-wave H36M fused kernel), H36M and CMU
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04n
mkdir -p $O
L=dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_ra35.so --config $cfg --rounds 7 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
