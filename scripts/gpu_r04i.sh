#!/bin/bash
# round 4 (r04i): forward parity suite; same-box A/B of HEAD against the
# previous commit (prev): E / F rows of the temporal tanh operand skewed by 32
# floats every other 16 rows (LDS bank conflicts of the fragment reads) --
# B=256 at H36M / CMU / 3DPW, B=32; LDS counters of both.
cd "$(dirname "$0")/.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04i
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg B=256" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config $cfg --rounds 5 >> $O/ab.txt 2>&1 || exit 1
done
echo "# h36m B=32" >> $O/ab.txt
timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_prev.so $L/libdstd_gcn.so --config h36m --batch 32 --rounds 5 --steps 20 >> $O/ab.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
export TMPDIR=/tmp
for lib in libdstd_gcn_prev libdstd_gcn; do
  set="SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$O/pmc_$lib/pmc1" -o run -- python3 $R/scripts/ab_kernels.py $R/$L/$lib.so --rounds 1 --steps 2 > "$O/pmc_$lib.log" 2>&1)
  st3=$?; echo "pmc $lib exit $st3"; [ $st3 -eq 0 ] || exit $st3
  python3 scripts/pmc_summary.py $O/pmc_$lib > $O/pmc_$lib.txt; grep -A1 "temporal_fused<35, 22, 1\|k_adj_hl<0, 35" $O/pmc_$lib.txt | cut -c1-700
done
