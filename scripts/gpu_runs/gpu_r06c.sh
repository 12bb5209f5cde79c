#!/bin/bash
# round 6 (r06c): (1) parity suite, then the experimental whole-model launch
# (DSTD_FWD_WHOLE_MODEL, k_model_fused) against the per-block schedule
# (scripts/mf_debug.py), (2) phase timeline of the fused block body (stamps
# build), (3) A/B at H36M / CMU / 3DPW B=256: new (k_block_fused per block),
# bfaux0 (h / P-Q stores with the default cache policy instead of sc1), nobf
# (round 5's two launches per block), (4) the training suite (agg_bwd
# 16-channel retry), (5) the gradient bar calibration
# (scripts/grad_bar_calibration.py)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06c
mkdir -p $O
L=$R/dstd-gcn_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -3 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -u scripts/mf_debug.py > $O/mf_debug.txt 2>&1; cat $O/mf_debug.txt
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so --config cmu >> $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_bfaux0.so \
    $L/libdstd_gcn_nobf.so --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; tail -4 $O/ab_$cfg.txt
done
unset DSTD_AB_FOREIGN_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -3 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
timeout -k 10 900 python -u scripts/grad_bar_calibration.py $O/grad_bar_calibration.json > $O/grad_bar.txt 2>&1
st=$?; tail -5 $O/grad_bar.txt; exit $st
