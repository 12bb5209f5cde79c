#!/bin/bash
# round 6 (r06c): (1) phase timeline of k_block_fused (stamps build), (2) A/B
# of the fused block's h / P-Q store policy (sc1 write-through vs default:
# bfaux0) against the two-launch schedule (nobf), (3) the training suite
# (agg_bwd 16-channel retry, dstd_debug_aggb_last tests), (4) the gradient bar
# calibration (scripts/grad_bar_calibration.py)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06c
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so --config cmu >> $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
for cfg in h36m cmu; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_bfaux0.so $L/libdstd_gcn_nobf.so \
    --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; tail -3 $O/ab_$cfg.txt
done
unset DSTD_AB_FOREIGN_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -3 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
timeout -k 10 900 python -u scripts/grad_bar_calibration.py profiles/r06c_grad_bar_calibration.json > $O/grad_bar.txt 2>&1
st=$?; cp profiles/r06c_grad_bar_calibration.json $O/ 2>/dev/null; tail -5 $O/grad_bar.txt; exit $st
