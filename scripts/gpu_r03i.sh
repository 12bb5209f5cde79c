#!/bin/bash
# round 3: next block's spatial adjacency in k_temporal_fused (phase 3):
# outputs vs the unfused path, A/B per kernel family, GPU suite; bisection of
# the fused-spatial output difference (sfm*: fused spatial on one (Cin, Cout) only)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in h36m cmu 3dpw; do
  timeout -k 10 180 python scripts/model_ab.py --config $c libdstd_gcn_nofused.so libdstd_gcn_nosfused.so libdstd_gcn_spre.so libdstd_gcn.so 2>&1 | grep -v amdgpu.ids || exit 1
done
DSTD_AB_FOREIGN_LIB=1 timeout -k 10 180 python scripts/model_ab.py --config h36m libdstd_gcn_nosfused.so libdstd_gcn_sfm1.so libdstd_gcn_sfm2.so libdstd_gcn_sfm4.so 2>&1 | grep -v amdgpu.ids || exit 1
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_nosfused.so dstd-gcn_amd/libdstd_gcn_spre.so dstd-gcn_amd/libdstd_gcn.so --config $c --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03i_pytest.txt 2>&1 || { tail -40 gpurun_out/r03i_pytest.txt; exit 1; }
tail -2 gpurun_out/r03i_pytest.txt
