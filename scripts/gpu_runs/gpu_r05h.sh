#!/bin/bash
# round 5 (r05h): E/F row placement (dstd_hilo.h EfRows) and the phase-1
# 16-byte plane stores against the round-4 layout (libdstd_gcn_efplain.so:
# -DDSTD_EF_PLAIN -DDSTD_TF_ST64) and E/F alone (libdstd_gcn_st64.so):
# outputs bit-identical, per-kernel-family A/B, LDS counters
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
for c in h36m cmu 3dpw; do
  timeout -k 10 200 python -u scripts/model_ab.py --config $c --batch 256 libdstd_gcn_efplain.so libdstd_gcn_st64.so libdstd_gcn.so > $O/bitid_$c.log 2>&1
  st=$?; tail -2 $O/bitid_$c.log; [ $st -eq 0 ] || exit $st
done
for c in h36m cmu 3dpw; do
  timeout -k 10 300 python -u scripts/ab_kernels.py dstd-gcn_amd/libdstd_gcn_efplain.so dstd-gcn_amd/libdstd_gcn_st64.so dstd-gcn_amd/libdstd_gcn.so --rounds 5 --config $c > $O/ab_$c.log 2>&1
  st=$?; echo "== $c"; cat $O/ab_$c.log; [ $st -eq 0 ] || exit $st
done
for v in efplain:libdstd_gcn_efplain.so st64:libdstd_gcn_st64.so new:libdstd_gcn.so; do
  PROF_TAG=r05h/pmc_${v%%:*} PMC_LIBS="${v#*:}" PMC_SETS="SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU" bash scripts/pmc_ab.sh
  st=$?; [ $st -eq 0 ] || exit $st
  echo "## ${v%%:*}" >> $O/pmc_summary.txt
  python3 scripts/pmc_summary.py $O/pmc_${v%%:*} >> $O/pmc_summary.txt
done
grep -A1 "^##\|temporal_fused<35, 22, 1, 64>\|k_adj_hl<0, 35, 70, 22>" $O/pmc_summary.txt
# training: float4 BatchNorm applies (libdstd_gcn.so) against the scalar loops
# (libdstd_gcn_bnscalar.so, -DDSTD_BN_NOVEC); two interleaved rounds, B=32 and 256
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for v in bnscalar:dstd-gcn_amd/libdstd_gcn_bnscalar.so new:dstd-gcn_amd/libdstd_gcn.so; do
    for B in 32 256; do
      DSTD_LIB=$R/${v#*:} timeout -k 10 200 python -u scripts/train_ab.py $B ${v%%:*} >> $O/train_ab.txt 2>&1
      st=$?; [ $st -eq 0 ] || { tail -5 $O/train_ab.txt; exit $st; }
    done
  done
done
grep -o '^[a-z0-9]* {"workload": "[^"]*B=[0-9]*\|"ms_per_step": [0-9.]*\|"host_issue_us_per_step": [0-9.]*' $O/train_ab.txt | paste - - - -
