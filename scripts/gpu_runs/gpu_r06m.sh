#!/bin/bash
# round 6 (r06m): is phase 3 bound by its plane stores?  Timeline with and
# without the stores (p3nsst: stores dropped, timing only) and the forward A/B
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06m
mkdir -p $O
L=$R/dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_stamps.so > $O/bf_timeline.txt 2>&1 || exit 1
cat $O/bf_timeline.txt
timeout -k 10 200 python -u scripts/bf_timeline.py $L/libdstd_gcn_p3nsst.so > $O/bf_timeline_nostore.txt 2>&1 || exit 1
cat $O/bf_timeline_nostore.txt
timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_p3ns.so \
    --config h36m --rounds 5 --steps 20 > $O/ab_h36m.txt 2>&1 || exit 1
grep wall $O/ab_h36m.txt | tail -2
