#!/bin/bash
# round 3: bench line (drop-in timing + side legs) and a kernel-stats profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { tail -20 gpurun_out/r03b_bench.err; exit 1; }
cat gpurun_out/r03b_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03b_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variant --no-side > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r03b_prof -name "*kernel_stats.csv" | head -3
