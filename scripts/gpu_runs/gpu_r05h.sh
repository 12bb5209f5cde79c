#!/bin/bash
# round 5 (r05h): E/F row placement (dstd_hilo.h EfRows) and the phase-1
# 16-byte plane stores against the round-4 layout (libdstd_gcn_efplain.so:
# -DDSTD_EF_PLAIN -DDSTD_TF_ST64) and E/F alone (libdstd_gcn_st64.so); the
# T=75 u-chunked fused temporal kernel against the unfused pair
# (libdstd_gcn_notf75.so, -DDSTD_NO_TF75): forward parity suite, outputs
# bit-identical, per-kernel-family A/B, LDS counters
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -2 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
for c in h36m cmu 3dpw; do
  timeout -k 10 200 python -u scripts/model_ab.py --config $c --batch 256 libdstd_gcn_efplain.so libdstd_gcn_st64.so libdstd_gcn.so > $O/bitid_$c.log 2>&1
  st=$?; tail -2 $O/bitid_$c.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 200 python -u scripts/model_ab.py --config h36m75 --batch 256 libdstd_gcn_notf75.so libdstd_gcn.so > $O/bitid_h36m75.log 2>&1
st=$?; tail -2 $O/bitid_h36m75.log; [ $st -eq 0 ] || exit $st
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python -u scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_efplain.so dstd-gcn_amd/libdstd_gcn_st64.so dstd-gcn_amd/libdstd_gcn.so --rounds 5 --config $c > $O/ab_$c.log 2>&1
  st=$?; echo "== $c"; cat $O/ab_$c.log; [ $st -eq 0 ] || exit $st
done
timeout -k 10 300 python -u scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_notf75.so dstd-gcn_amd/libdstd_gcn.so --rounds 4 --config h36m75 > $O/ab_h36m75.log 2>&1
st=$?; echo "== h36m75"; cat $O/ab_h36m75.log; [ $st -eq 0 ] || exit $st
for v in efplain:libdstd_gcn_efplain.so st64:libdstd_gcn_st64.so new:libdstd_gcn.so; do
  PROF_TAG=r05h/pmc_${v%%:*} PMC_LIBS="${v#*:}" PMC_SETS="SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU" bash scripts/pmc_ab.sh
  st=$?; [ $st -eq 0 ] || exit $st
  echo "## ${v%%:*}" >> $O/pmc_summary.txt
  python3 scripts/pmc_summary.py $O/pmc_${v%%:*} >> $O/pmc_summary.txt
done
grep -A1 "^##\|temporal_fused<35, 22, 1, 64>\|k_adj_hl<0, 35, 70, 22>" $O/pmc_summary.txt
