#!/bin/bash
# round 6 (r06j): phase-2 stage loads issued before the phase-1 barrier (load/store split)
# on top of phase 3 with 2 column tiles per task -- parity, timeline, A/B against
# the split with TPI 1 (sp1), no split with TPI 2 / 1 (ns2 / ns1) and bf0
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06j
mkdir -p $O
L=$R/dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -3 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_sp1.so $L/libdstd_gcn_ns2.so $L/libdstd_gcn_ns1.so $L/libdstd_gcn_bf0.so \
    --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; tail -3 $O/ab_$cfg.txt
done
