#!/bin/bash
# round 3 (r03s): aggregation kernels -- microbenchmark per form, GPU training
# tests, training-step A/B against the strided GEMMs
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/r03s
AGG_CASES="${AGG_CASES:-2:0 0:0 3:0}" bash scripts/gpu_micro_agg.sh || exit 1
cp gpurun_out/agg/micro.txt gpurun_out/r03s/micro.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r03s/pytest_train.log 2>&1
st=$?; tail -3 gpurun_out/r03s/pytest_train.log; [ $st -eq 0 ] || exit $st
for i in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 slab >> gpurun_out/r03s/ab.txt 2>&1 || exit 1
  DSTD_TRAIN_AGG_GEMM=1 timeout -k 10 200 python -u scripts/train_ab.py 32 gemm >> gpurun_out/r03s/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r03s/ab.txt | cut -c1-60,150-400
