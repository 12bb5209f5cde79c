#!/bin/bash
# round 3: GPU suite (incl. the 2-process native DP tests), then the bench line
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 180 --timeout-method thread > gpurun_out/r03c_pytest.txt 2>&1 || { tail -40 gpurun_out/r03c_pytest.txt; exit 1; }
tail -3 gpurun_out/r03c_pytest.txt
grep "gradient error / fp32 noise" gpurun_out/r03c_pytest.txt
bash scripts/gpu_r03b.sh
