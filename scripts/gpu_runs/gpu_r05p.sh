#!/bin/bash
# round 5 (r05p): spatial static priority now default (nosp = off): parity
# suite; the same for k_temporal_hl (th256) and k_adj_hl (adj384) at B=32
# and T=75 where those run; host cost per launch (scripts/micro/launch_cost);
# kernel trace of the B=32 training step
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -1 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
timeout -k 10 60 ./scripts/micro/launch_cost | tee $O/launch_cost.txt || exit 1
L="libdstd_gcn_nosp.so libdstd_gcn.so libdstd_gcn_th256.so libdstd_gcn_adj384.so"
timeout -k 10 200 python -u scripts/model_ab.py --config h36m --batch 32 $L > $O/bitid_h36m32.log 2>&1
st=$?; tail -3 $O/bitid_h36m32.log; [ $st -eq 0 ] || exit $st
LP=$(for l in $L; do echo -n "dstd-gcn_amd/$l "; done)
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 5 --config h36m --batch 32 --steps 40 > $O/ab_h36m_b32.log 2>&1
st=$?; echo "== h36m B=32"; cat $O/ab_h36m_b32.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 4 --config h36m75 > $O/ab_h36m75.log 2>&1
st=$?; echo "== h36m75"; cat $O/ab_h36m75.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u scripts/ab_kernels.py $LP --rounds 4 --config h36m > $O/ab_h36m.log 2>&1
st=$?; echo "== h36m"; cat $O/ab_h36m.log; [ $st -eq 0 ] || exit $st
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trt -o tr -- python3 scripts/bench_train.py --batch 32 --steps 10 --warmup 3 > $O/trt.log 2>&1 || exit 1
f=$(find $O/trt -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_summary.py "$f" 3 40 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt || exit 1
head -40 $O/train_trace_summary.txt
