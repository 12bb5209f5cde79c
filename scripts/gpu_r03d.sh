#!/bin/bash
# round 3: GPU suite + A/B of the batched-prologue library against the
# previous revision, then the bench line
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 180 --timeout-method thread > gpurun_out/r03d_pytest.txt 2>&1 || { tail -40 gpurun_out/r03d_pytest.txt; exit 1; }
tail -2 gpurun_out/r03d_pytest.txt
grep "gradient error / fp32 noise" gpurun_out/r03d_pytest.txt
export DSTD_AB_FOREIGN_LIB=1
for c in h36m cmu 3dpw; do
  timeout -k 10 240 python scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_prev.so dstd-gcn_amd/libdstd_gcn.so --config $c --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done
unset DSTD_AB_FOREIGN_LIB
bash scripts/gpu_r03b.sh
