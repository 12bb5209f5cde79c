#!/bin/bash
# round 3: phase 3 v2 (weights in LDS, one tile space): timeline, outputs, A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/timeline.py dstd-gcn_amd/libdstd_gcn_stamps.so --hl 2>&1 | grep -v amdgpu.ids || exit 1
for c in h36m cmu 3dpw; do
  timeout -k 10 180 python scripts/model_ab.py --config $c libdstd_gcn_nofused.so libdstd_gcn_nosfused.so libdstd_gcn_spre.so libdstd_gcn.so 2>&1 | grep -v amdgpu.ids || exit 1
done
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_nosfused.so dstd-gcn_amd/libdstd_gcn_spre.so dstd-gcn_amd/libdstd_gcn.so --config $c --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done
