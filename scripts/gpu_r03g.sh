#!/bin/bash
# round 3: phase-serial fused spatial kernel -- whole-model outputs vs the
# unfused path (expected bit-identical), GPU suite, A/B per kernel family
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in h36m cmu 3dpw; do
  timeout -k 10 180 python scripts/model_ab.py --config $c libdstd_gcn_nofused.so libdstd_gcn.so libdstd_gcn_nosfused.so 2>&1 | grep -v amdgpu.ids || exit 1
done
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_nofused.so dstd-gcn_amd/libdstd_gcn_nosfused.so dstd-gcn_amd/libdstd_gcn.so --config $c --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03g_pytest.txt 2>&1 || { tail -40 gpurun_out/r03g_pytest.txt; exit 1; }
tail -2 gpurun_out/r03g_pytest.txt
