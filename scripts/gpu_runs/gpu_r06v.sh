#!/bin/bash
# round 6 (r06v): H36M block kernel at 8 waves (two per SIMD, as CMU / 3DPW)
# against the default 12, with round 5's two-launch schedule beside them
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06v
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "block_fused and h36m" > $O/pytest.log 2>&1
timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_nw8.so $L/libdstd_gcn_nobf.so \
    --config h36m --rounds 9 --steps 20 > $O/ab_h36m.txt 2>&1 || exit 1
grep wall $O/ab_h36m.txt | tail -3
