#!/bin/bash
# round 4 (r04h): same-box forward A/B of HEAD against tsc (the separable
# tanh's two FMAs as scalar v_fma_f32 instead of one v_pk_fma_f32 pair:
# packed f32 beside MFMAs is an issue-cost anti-lever per the MI355X guide),
# B=256 H36M / CMU / 3DPW; B=32 training step with the fused Adam.
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04h
mkdir -p $O
L=dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_tsc.so --config $cfg --rounds 5 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
unset DSTD_AB_FOREIGN_LIB
timeout -k 10 300 python -u scripts/bench_train.py --batch 32 > $O/train.log 2>&1; st=$?
grep metric $O/train.log | cut -c1-300; exit $st
