#!/bin/bash
# round 3: fused spatial chunking experiments (F = 18/9/14 default, 16, 8;
# phase 2 alone, phase 1 alone) and the plane parity pattern of one block
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/tf_debug.py b_64_64_h36m libdstd_gcn_nosfused.so libdstd_gcn.so 2>&1 | grep -v amdgpu.ids || exit 1
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_nosfused.so dstd-gcn_amd/libdstd_gcn.so dstd-gcn_amd/libdstd_gcn_sff16.so dstd-gcn_amd/libdstd_gcn_sff8.so dstd-gcn_amd/libdstd_gcn_sfnoprod.so dstd-gcn_amd/libdstd_gcn_sfnocons.so --config $c --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
