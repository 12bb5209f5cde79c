#!/bin/bash
# round 3 (r03u): skinny GEMM kernels -- GPU suite, training-step A/B
# (default / DSTD_GEMM_GENERIC=1 / + DSTD_TRAIN_AGG_GEMM=1), kernel trace
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${R03U_TESTS:-tests/} > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
for i in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 skinny >> $O/ab.txt 2>&1 || exit 1
  DSTD_GEMM_GENERIC=1 timeout -k 10 200 python -u scripts/train_ab.py 32 generic >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-10,130-400
bash scripts/gpu_r03t.sh > $O/trace.txt 2>&1; st=$?
head -30 $O/trace.txt; exit $st
