#!/bin/bash
# round 4 (r04g): forward parity suite, then same-box A/B of HEAD against the
# previous commit (prev): four-chain range maxima (fewer hazard s_nops) and
# the adjacency kernel's column chunks spread over more workgroups below one
# (sample, graph) set per CU -- B=256 at H36M / CMU / 3DPW and B=32 at H36M.
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04g
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config $cfg --rounds 5 >> $O/ab.txt 2>&1 || exit 1
done
for B in 32 64; do
  echo "# h36m B=$B" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config h36m --batch $B --rounds 5 --steps 20 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
