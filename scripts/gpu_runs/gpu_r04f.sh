#!/bin/bash
# round 4 (r04f): SyncBN test (tail held to the single-process step's);
# forward + training A/B of a build without SLP vectorisation (noslp: the
# compiler's packed-f32 v_pk_* pairs, an issue-cost anti-lever beside MFMAs
# per the MI355X guide); LDS / VALU counters per fused-kernel phase through
# builds that skip phase 1 (skp1) or phase 2 (skp2).
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04f
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1
st=$?; grep -E "median|passed|failed|Error" $O/pytest_dist.log | cut -c1-600 | tail -8
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_noslp.so --config $cfg --rounds 5 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-330
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_noslp; do
    DSTD_LIB="$R/$L/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 > $O/train_$lib.$r.log 2>&1
    st2=$?; echo "$lib round $r exit $st2"; grep metric $O/train_$lib.$r.log | cut -c1-300; [ $st2 -eq 0 ] || exit $st2
  done
done
export TMPDIR=/tmp
for lib in libdstd_gcn libdstd_gcn_skp1 libdstd_gcn_skp2 libdstd_gcn_noslp; do
  set="SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$O/pmc_$lib/pmc1" -o run -- python3 $R/scripts/ab_kernels.py $R/$L/$lib.so --rounds 1 --steps 2 > "$O/pmc_$lib.log" 2>&1)
  st3=$?; echo "pmc $lib exit $st3"; [ $st3 -eq 0 ] || exit $st3
  python3 scripts/pmc_summary.py $O/pmc_$lib > $O/pmc_$lib.txt; grep -A1 "temporal_fused<35, 22, 1\|spatial_hl<22, 64, 64" $O/pmc_$lib.txt | cut -c1-700
done
exit $st
