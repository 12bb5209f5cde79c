#!/bin/bash
# round 5 (r05o): static VALU-arbitration priority for the younger waves
# (MI355X guide T5 static form) in k_spatial_hl (waves 4-7: sp256) and
# k_temporal_fused (waves 4-11: tf256; 8-11: tf512; both = sp256 + tf512):
# outputs bit-identical, per-kernel-family A/B at B=256 (h36m, 3dpw) and B=32
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05o
mkdir -p $O
L="libdstd_gcn.so libdstd_gcn_sp256.so libdstd_gcn_tf256.so libdstd_gcn_tf512.so libdstd_gcn_both.so"
timeout -k 10 200 python -u scripts/model_ab.py --config h36m --batch 256 $L > $O/bitid_h36m.log 2>&1
st=$?; tail -4 $O/bitid_h36m.log; [ $st -eq 0 ] || exit $st
LP=$(for l in $L; do echo -n "dstd-gcn_amd/$l "; done)
for c in h36m 3dpw; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config $c > $O/ab_$c.log 2>&1
  st=$?; echo "== $c"; cat $O/ab_$c.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config h36m --batch 32 --steps 40 > $O/ab_h36m_b32.log 2>&1
st=$?; echo "== h36m B=32"; cat $O/ab_h36m_b32.log; [ $st -eq 0 ] || exit $st
