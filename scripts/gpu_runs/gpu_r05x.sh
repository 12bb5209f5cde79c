#!/bin/bash
# round 5 (r05x): three waves per SIMD in k_spatial_hl with the youngest third
# (w3p512) or two thirds (w3p256) at priority 1, and the younger waves'
# priority during the fused temporal kernel's units only (tfp2: waves 4-11,
# tfp2b: 8-11): outputs bit-identical, per-family A/B at B=256 (h36m, 3dpw,
# cmu) and B=32
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05x
mkdir -p $O
L="libdstd_gcn.so libdstd_gcn_w3p512.so libdstd_gcn_w3p256.so libdstd_gcn_tfp2.so libdstd_gcn_tfp2b.so"
timeout -k 10 200 python -u scripts/model_ab.py --config h36m --batch 256 $L > $O/bitid_h36m.log 2>&1
st=$?; tail -4 $O/bitid_h36m.log; [ $st -eq 0 ] || exit $st
LP=$(for l in $L; do echo -n "dstd-gcn_amd/$l "; done)
for c in h36m 3dpw cmu; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config $c > $O/ab_$c.log 2>&1
  st=$?; echo "== $c"; grep -v amdgpu.ids $O/ab_$c.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 4 --config h36m --batch 32 --steps 40 > $O/ab_h36m_b32.log 2>&1
st=$?; echo "== h36m B=32"; grep -v amdgpu.ids $O/ab_h36m_b32.log; [ $st -eq 0 ] || exit $st
