#!/bin/bash
# round 4 (r04v): streaming GEMM and adjacency column blocks now on by
# default -- the whole GPU suite on HEAD, then the streaming GEMM's item width
# (nt2: 32-column items, nt2n: without the next-item prefetch, nt4n: 64-column
# items without it) in the microbenchmark and the training step, against HEAD
# and the former defaults (off)
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; echo "suite: $(tail -1 $O/pytest_gpu.log)"; [ $st -eq 0 ] || exit $st
for v in off "" nt2 nt2n nt4n; do
  b=scripts/micro/skinny_micro${v:+_$v}
  timeout -k 10 60 $b > $O/micro_${v:-head}.txt 2>&1; st=$?
  echo "== ${v:-head} (exit $st): $(tail -1 $O/micro_${v:-head}.txt)"; [ $st -eq 0 ] || exit $st
done
export DSTD_AB_FOREIGN_LIB=1
for r in 1 2; do
  for lib in libdstd_gcn_off libdstd_gcn libdstd_gcn_nt2 libdstd_gcn_nt2n libdstd_gcn_nt4n; do
    DSTD_LIB="$R/dstd-gcn_amd/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-110; [ $st -eq 0 ] || exit $st
  done
done
# kernel trace of the B=32 step on HEAD (per-queue busy time: is the main
# stream waiting on the weight-gradient stream?)
unset DSTD_AB_FOREIGN_LIB
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tt" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 6 --warmup 3 > "$O/tt.log" 2>&1)
st=$?; echo "train trace exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary.txt; tail -3 $O/train_trace_summary.txt
