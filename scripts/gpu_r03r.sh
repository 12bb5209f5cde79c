#!/bin/bash
# round 3 (r03r): slab aggregation kernels for the training products -- GPU
# training tests, A/B against the strided GEMMs, kernel stats of one step
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/r03r
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r03r/pytest_train.log 2>&1
st=$?; tail -3 gpurun_out/r03r/pytest_train.log; [ $st -eq 0 ] || exit $st
for i in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 slab >> gpurun_out/r03r/ab.txt 2>&1 || exit 1
  DSTD_TRAIN_AGG_GEMM=1 timeout -k 10 200 python -u scripts/train_ab.py 32 gemm >> gpurun_out/r03r/ab.txt 2>&1 || exit 1
done
cat gpurun_out/r03r/ab.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r03r/kt" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/train_prof.py" 32 10 > "$GRAFT_REPO_ROOT/gpurun_out/r03r/kt.log" 2>&1
echo "kt exit $?"
