#!/bin/bash
# round 6 (r06u): the final block-kernel forward against round 5's two-launch
# schedule built from the same tree (-DDSTD_NO_BFUSED: k_adj_hl<0> +
# k_spatial_hl + k_temporal_fused per block, 15 launches), same box
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06u
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_nobf.so \
    --config $cfg --rounds 7 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; grep wall $O/ab_$cfg.txt | tail -2
done
