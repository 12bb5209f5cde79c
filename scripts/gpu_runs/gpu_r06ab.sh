#!/bin/bash
# round 6 (r06ab): VERDICT r05 item 8 -- a T = 75 lever on the unfused pair:
# column chunks per sample of the temporal adjacency launch (k_adj_hl<1>,
# DSTD_ADJ_T_NCHUNK 1 / 2 (default) / 3 / 4), at the T=75 variant's B=256 and
# at B=32 (the small-batch schedule uses the same kernel)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ab
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "h36m75 or ragged or small" > $O/pytest.log 2>&1
st=$?; tail -1 $O/pytest.log; [ $st -eq 0 ] || exit $st
timeout -k 10 500 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_tch1.so $L/libdstd_gcn_tch3.so $L/libdstd_gcn_tch4.so \
    --config h36m75 --rounds 5 --steps 10 > $O/ab_h36m75.txt 2>&1 || exit 1
grep wall $O/ab_h36m75.txt | tail -4
timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_tch1.so $L/libdstd_gcn_tch3.so $L/libdstd_gcn_tch4.so \
    --config h36m --batch 32 --rounds 5 --steps 50 > $O/ab_h36m_b32.txt 2>&1 || exit 1
grep wall $O/ab_h36m_b32.txt | tail -4
