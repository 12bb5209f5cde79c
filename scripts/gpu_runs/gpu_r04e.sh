#!/bin/bash
# round 4 (r04e): SyncBN test against the fp64 oracle; fused-kernel phase-1
# breakdown (stamps mode 4); VALU / MFMA / LDS counters of the forward, r03
# and HEAD in separate processes; kernel trace of the B=32 training step.
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04e
mkdir -p $O
L=dstd-gcn_amd
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1
st=$?; grep -E "median|passed|failed|Error" $O/pytest_dist.log | cut -c1-600 | tail -8
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 120 python -u scripts/timeline.py $L/libdstd_gcn_stamps.so --hl > $O/timeline.txt 2>&1; st2=$?
grep -v amdgpu.ids $O/timeline.txt | grep -v "XCC\|placement\|WG/CU"; [ $st2 -eq 0 ] || exit $st2
export TMPDIR=/tmp
for lib in libdstd_gcn_r03 libdstd_gcn; do
  i=0
  for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$O/pmc_$lib/pmc$i" -o run -- python3 $R/scripts/ab_kernels.py $R/$L/$lib.so --rounds 1 --steps 2 > "$O/pmc_$lib.$i.log" 2>&1)
    st3=$?; echo "pmc $lib pass $i exit $st3"; [ $st3 -eq 0 ] || exit $st3
  done
  python3 scripts/pmc_summary.py $O/pmc_$lib > $O/pmc_$lib.txt; grep -A1 "temporal_fused<35, 22, 1\|spatial_hl<22, 64, 64" $O/pmc_$lib.txt | cut -c1-900
done
unset DSTD_AB_FOREIGN_LIB
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tt" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 6 --warmup 3 > "$O/tt.log" 2>&1)
st4=$?; echo "train trace exit $st4"; [ $st4 -eq 0 ] || exit $st4
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 | tee $O/train_trace_summary.txt
exit $st
