#!/bin/bash
# round 5 (r05cc): end-of-round state (after the training changes of r05z / r05bb) --
# whole GPU suite, smoke, the bench line, kernel traces at B=256 / B=32 and
# of the B=32 training step (steady state, last 3 steps), HBM traffic passes
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r05cc
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
st=$?; tail -2 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; st=$?; grep -v amdgpu.ids $O/smoke.log | tail -3; [ $st -eq 0 ] || exit $st
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; st=$?
tail -c 600 $O/bench.json; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-variant --no-side > "$O/kt.log" 2>&1)
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/kstats.py $O/kt/run_kernel_stats.csv 13 12
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt32" -o run -- python3 "$R/bench.py" --batch 32 --steps 50 --warmup 5 --no-cpu-baseline --no-variant --no-side > "$O/kt32.log" 2>&1)
st=$?; echo "kt32 exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/kstats.py $O/kt32/run_kernel_stats.csv 105 12
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tt" -o run -- python3 "$R/scripts/bench_train.py" --batch 32 --steps 6 --warmup 3 > "$O/tt.log" 2>&1)
st=$?; echo "train trace exit $st"; [ $st -eq 0 ] || exit $st
python3 scripts/trace_summary.py $O/tt/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 | tee $O/train_trace_summary.txt
# HBM traffic of the forward kernels at HEAD (one counter per pass)
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$O/pmc$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-variant --no-side > "$O/pmc$i.log" 2>&1)
  st=$?; echo "pmc pass $i ($set) exit $st"; [ $st -eq 0 ] || exit $st
done
