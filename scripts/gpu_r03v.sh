#!/bin/bash
# round 3 (r03v): kernel-generation retirement + training GEMM epilogues --
# GPU suite, skinny micro, training A/B, full bench line
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 60 scripts/micro/skinny_micro > $O/skinny_micro.txt 2>&1 || exit 1
DSTD_GEMM_GENERIC=1 timeout -k 10 60 scripts/micro/skinny_micro >> $O/skinny_micro.txt 2>&1 || exit 1
cat $O/skinny_micro.txt
for i in 1 2; do
  timeout -k 10 200 python -u scripts/train_ab.py 32 default >> $O/ab.txt 2>&1 || exit 1
  DSTD_GEMM_GENERIC=1 timeout -k 10 200 python -u scripts/train_ab.py 32 generic >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-10,130-300
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 1500 $O/bench.json; exit $st
