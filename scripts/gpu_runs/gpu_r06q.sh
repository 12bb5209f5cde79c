#!/bin/bash
# round 6 (r06q): phase 3's static prologue loads (images, Astat, bias) issued
# before the barrier that ends phase 2 (SAdjStatic) -- parity suite, timeline,
# A/B against the same tree without it (pl0)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06q
mkdir -p $O
L=$R/dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_pl0.so \
    --config $cfg --rounds 7 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; grep wall $O/ab_$cfg.txt | tail -2
done
