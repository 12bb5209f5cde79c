#!/bin/bash
# round 4 (r04af): records for the next round -- the B=32 training step's
# kernel trace on the final HEAD, and SQ counters of the streaming GEMM in the
# microbenchmark (where its time goes: MFMA vs VALU vs waits)
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04af
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tt" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 6 --warmup 3 > "$O/tt.log" 2>&1)
st=$?; echo "train trace exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt; head -2 $O/train_trace_summary.txt; tail -2 $O/train_trace_summary.txt
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$O/pmc" -o run -- "$R/scripts/micro/skinny_micro" > "$O/pmc.log" 2>&1)
st=$?; echo "pmc exit $st"; [ $st -eq 0 ] || exit $st
