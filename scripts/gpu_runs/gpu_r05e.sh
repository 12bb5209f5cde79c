#!/bin/bash
# round 5 (r05e): grad_tail_bisect.py with the worst block in detail
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u scripts/grad_tail_bisect.py > $O/grad_tail.txt 2>&1
st=$?; cat $O/grad_tail.txt | grep -v amdgpu.ids | tail -50; exit $st
