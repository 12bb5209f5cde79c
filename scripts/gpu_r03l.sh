#!/bin/bash
# round 3: device-side dropout seed + graphed training step -- train tests,
# then the training side leg of the bench (eager and graph replay)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r03l_train.txt 2>&1 || { tail -40 gpurun_out/r03l_train.txt; exit 1; }
tail -2 gpurun_out/r03l_train.txt
timeout -k 10 200 python -c "
import sys, json, torch
sys.path[:0] = ['.', 'dstd-gcn_amd']
import bench
print(json.dumps(bench.train_leg(torch.device('cuda', 0), 32, 20, 5)))
" 2>&1 | grep -v amdgpu.ids
