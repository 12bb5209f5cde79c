#!/bin/bash
# Copy one GPU run's results (gpurun_out/<tag>) into profiles/<tag>_*:
# bench line, kernel stats at B=256 / B=32, training trace summary, HBM
# traffic (scripts/pmc_traffic.py -> profiles/pmc_traffic.json).
#   scripts/save_profiles.sh r04s
set -e
cd "$(dirname "$0")/.."
T=$1
G=gpurun_out/$T
[ -d "$G" ] || { echo "no $G"; exit 1; }
[ -f $G/bench.json ] && tail -1 $G/bench.json > profiles/${T}_bench.json
[ -f $G/kt/run_kernel_stats.csv ] && cp $G/kt/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
[ -f $G/kt32/run_kernel_stats.csv ] && cp $G/kt32/run_kernel_stats.csv profiles/${T}_kernel_stats_b32.csv
if [ -f $G/train_trace_summary.txt ]; then
  { echo "# ($T): kernel trace of the B=32 3DPW training step (scripts/bench_train.py), last 3 steady-state steps"; cat $G/train_trace_summary.txt; } > profiles/${T}_train_trace_summary.txt
fi
if [ -d $G/pmc1 ] && [ -d $G/pmc2 ]; then
  python3 scripts/pmc_traffic.py $G profiles/${T}
fi
ls -la profiles/${T}_* profiles/pmc_traffic.json 2>/dev/null
