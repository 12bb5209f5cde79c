#!/bin/bash
# round 5 (r05j): where the training step's host time goes -- per-phase host
# time from an idle queue (scripts/train_host_probe.py, fused Adam), then the
# HIP API trace of bench_train's B=32 steps (per-call host cost of each API)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05j
mkdir -p $O
timeout -k 10 300 python -u scripts/train_host_probe.py > $O/host_probe.txt 2>&1
st=$?; cat $O/host_probe.txt | grep -v amdgpu; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$O/ht" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 10 --warmup 3 > "$O/ht.log" 2>&1)
st=$?; echo "hip trace exit $st"; [ $st -eq 0 ] || exit $st
ls $O/ht
head -25 $O/ht/run_hip_api_stats.csv
