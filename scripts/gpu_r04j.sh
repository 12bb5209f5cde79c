#!/bin/bash
# round 4 (r04j): forward parity suite; same-box A/B of HEAD against the
# previous commit (prev): phase 3's constants (conv_rm images, Astat table,
# bias) loaded across the barrier that waits for the sample's last GC unit
cd "$(dirname "$0")/.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04j
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config $cfg --rounds 7 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
