#!/bin/bash
# round 3 (r03t): kernel trace of the B=32 training step
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/r03t
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03t/kt" -o run -- python3 "$R/scripts/train_prof.py" 32 10 > "$R/gpurun_out/r03t/kt.log" 2>&1
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
python3 "$R/scripts/trace_summary.py" "$R/gpurun_out/r03t/kt/run_kernel_trace.csv" 10 40
