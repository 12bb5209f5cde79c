#!/bin/bash
# round 3: phase 3 with per-graph tanh path -- GPU suite, A/B against the
# separate-adjacency schedule (nospre build), bench line and kernel stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 180 --timeout-method thread > gpurun_out/r03m_pytest.txt 2>&1 || { tail -40 gpurun_out/r03m_pytest.txt; exit 1; }
tail -2 gpurun_out/r03m_pytest.txt

timeout -k 10 400 python bench.py > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err || { tail -20 gpurun_out/r03m_bench.err; exit 1; }
cat gpurun_out/r03m_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03m_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variant --no-side > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r03m_prof -name "*kernel_stats.csv" | head -3
