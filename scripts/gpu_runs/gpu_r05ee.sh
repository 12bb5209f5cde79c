#!/bin/bash
# round 5 (r05ee): small-batch adjacency chunking (k_adj_hl below one set per
# CU): p75 / p50 / p0 = chunks aimed at 75% / 50% / 0% of the CUs (the
# kernel floor NCHUNK) instead of 100%; r05ee first pass: more chunks lost;
# B=32 / B=64 forward A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05ee
mkdir -p $O
L="libdstd_gcn.so libdstd_gcn_p75.so libdstd_gcn_p50.so libdstd_gcn_p0.so"
timeout -k 10 200 python -u scripts/model_ab.py --config h36m --batch 32 $L > $O/bitid_h36m32.log 2>&1
st=$?; tail -3 $O/bitid_h36m32.log; [ $st -eq 0 ] || exit $st
LP=$(for l in $L; do echo -n "dstd-gcn_amd/$l "; done)
for b in 32 64; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config h36m --batch $b --steps 40 > $O/ab_h36m_b$b.log 2>&1
  st=$?; echo "== h36m B=$b"; grep -v amdgpu.ids $O/ab_h36m_b$b.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 4 --config 3dpw --batch 32 --steps 40 > $O/ab_3dpw_b32.log 2>&1
st=$?; echo "== 3dpw B=32"; grep -v amdgpu.ids $O/ab_3dpw_b32.log; [ $st -eq 0 ] || exit $st
