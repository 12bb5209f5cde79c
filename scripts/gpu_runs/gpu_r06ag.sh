#!/bin/bash
# round 6 (r06ag): non-temporal (nt) loads for the last read of the h rows
# (hnt), of the encoder residual (rnt), both (hrnt) in the joint units
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ag
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_hnt.so $L/libdstd_gcn_rnt.so $L/libdstd_gcn_hrnt.so \
    --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; grep wall $O/ab_$cfg.txt | tail -4
done
