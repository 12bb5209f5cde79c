#!/bin/bash
# round 3: GPU suite on the fixed library, fused-temporal variants vs the
# unfused path, A/B of the variants (one GPU step per line, each bounded)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_pytest.txt 2>&1 || { tail -30 gpurun_out/r03a_pytest.txt; exit 1; }
tail -3 gpurun_out/r03a_pytest.txt
for b in b_64_64_h36m b_64_64_cmu; do
  timeout -k 10 120 python scripts/tf_debug.py $b libdstd_gcn.so libdstd_gcn_hoist.so libdstd_gcn_tpi2.so libdstd_gcn_tpi2hoist.so 2>&1 | grep rel >> gpurun_out/r03a_variants.txt || exit 1
done
for c in h36m cmu 3dpw; do
  timeout -k 10 240 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn.so dstd-gcn_amd/libdstd_gcn_hoist.so dstd-gcn_amd/libdstd_gcn_tpi2.so dstd-gcn_amd/libdstd_gcn_tpi2hoist.so --config $c --rounds 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r03a_variants.txt || exit 1
done
cat gpurun_out/r03a_variants.txt
