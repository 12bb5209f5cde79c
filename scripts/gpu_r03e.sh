#!/bin/bash
# round 3: the pipelined temporal kernel -- parity vs the unfused path, GPU
# suite, A/B against k_temporal_fused
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for b in b_64_64_h36m b_64_64_cmu; do
  timeout -k 10 120 python scripts/tf_debug.py $b libdstd_gcn.so libdstd_gcn_pipetpi2.so libdstd_gcn_fusedold.so 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03e_pytest.txt 2>&1 || { tail -40 gpurun_out/r03e_pytest.txt; exit 1; }
tail -2 gpurun_out/r03e_pytest.txt
for c in h36m cmu 3dpw; do
  timeout -k 10 240 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_fusedold.so dstd-gcn_amd/libdstd_gcn.so dstd-gcn_amd/libdstd_gcn_pipetpi2.so --config $c --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done
