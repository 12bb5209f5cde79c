#!/bin/bash
# round 5 (r05dd): k_spatial_hl variants on top of the younger-half priority:
# the identity residual loaded after the aggregations (splate), priority for
# waves 6-7 only (sp384) or 2-7 (sp128): bit-identical, per-family A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05dd
mkdir -p $O
L="libdstd_gcn.so libdstd_gcn_splate.so libdstd_gcn_sp384.so libdstd_gcn_sp128.so"
timeout -k 10 200 python -u scripts/model_ab.py --config h36m --batch 256 $L > $O/bitid_h36m.log 2>&1
st=$?; tail -4 $O/bitid_h36m.log; [ $st -eq 0 ] || exit $st
LP=$(for l in $L; do echo -n "dstd-gcn_amd/$l "; done)
for c in h36m 3dpw cmu; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config $c > $O/ab_$c.log 2>&1
  st=$?; echo "== $c"; grep -v amdgpu.ids $O/ab_$c.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 4 --config h36m --batch 32 --steps 40 > $O/ab_h36m_b32.log 2>&1
st=$?; echo "== h36m B=32"; grep -v amdgpu.ids $O/ab_h36m_b32.log; [ $st -eq 0 ] || exit $st
