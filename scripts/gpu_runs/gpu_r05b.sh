#!/bin/bash
# round 5 (r05b): the whole-model gradient tail bisected per block, the
# fp64 conditioning and the fp32 noise distribution (scripts/grad_tail_bisect.py)
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u scripts/grad_tail_bisect.py > $O/grad_tail.txt 2>&1
st=$?; cat $O/grad_tail.txt | grep -v amdgpu.ids | tail -40; exit $st
