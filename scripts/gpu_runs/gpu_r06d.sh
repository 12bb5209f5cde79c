#!/bin/bash
# round 6 (r06d): the experimental whole-model launch with an L1 invalidate
# at every block start -- correctness against the per-block schedule
# (scripts/mf_debug.py), then its time against it (scripts/flag_ab.py,
# interleaved, one library) at H36M / CMU / 3DPW B=256
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r06d
mkdir -p $O
timeout -k 10 200 python -u scripts/mf_debug.py > $O/mf_debug.txt 2>&1 || exit 1
cat $O/mf_debug.txt
for cfg in h36m cmu 3dpw; do
  timeout -k 10 300 python -u scripts/flag_ab.py --config $cfg default=0 whole=32 > $O/flag_ab_$cfg.txt 2>&1 || exit 1
  grep median $O/flag_ab_$cfg.txt
done
