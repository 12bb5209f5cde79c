#!/bin/bash
# round 6 (r06t): probe -- the B=256 forward as 2 or 4 concurrent sub-batches
# on their own HIP streams (block kernel forced per sub-batch)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06t
mkdir -p $O
for cfg in h36m 3dpw; do
  timeout -k 10 300 python -u scripts/stream_split_probe.py --config $cfg --rounds 5 --steps 20 > $O/probe_$cfg.txt 2>&1 || exit 1
  cat $O/probe_$cfg.txt
done
