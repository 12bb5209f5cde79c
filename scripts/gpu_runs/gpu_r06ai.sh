#!/bin/bash
# round 6 (r06ai): per-phase timeline of the final tree's H36M encoder block
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06ai
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $R/dstd-gcn_amd/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
