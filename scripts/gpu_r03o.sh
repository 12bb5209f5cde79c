#!/bin/bash
# round 3: training GEMM k_gemm2 -- training tests, step time A/B against the
# k_gemm build, kernel stats of the step
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r03o_train.txt 2>&1 || { tail -40 gpurun_out/r03o_train.txt; exit 1; }
tail -2 gpurun_out/r03o_train.txt
for lib in libdstd_gcn_gemmv1.so libdstd_gcn.so; do
  DSTD_LIB=$GRAFT_REPO_ROOT/dstd-gcn_amd/$lib timeout -k 10 200 python -c "
import sys, json, torch
sys.path[:0] = ['.', 'dstd-gcn_amd']
import bench
r = bench.train_leg(torch.device('cuda', 0), 32, 20, 5)
print('$lib', json.dumps({k: r[k] for k in ('ms_per_step', 'host_us_per_step')}), json.dumps(r['graph_replay']))
" 2>&1 | grep -v amdgpu.ids || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03o_trainprof -o run -- python3 $GRAFT_REPO_ROOT/scripts/train_prof.py 32 10 > /dev/null 2>&1 || exit 1
