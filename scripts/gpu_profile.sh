#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then PMC counters in
# separate passes (never combined with other trace domains).
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/${PROF_TAG:-prof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 2
BENCH="$REPO/bench.py ${PROF_BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-variant --no-side}"

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $BENCH > "$OUT/kt.log" 2>&1
st=$?; echo "kernel-trace exit $st"; [ $st -eq 0 ] || exit $st
if [ -n "${PROF_LIST:-}" ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; fi
i=0
for set in ${PROF_PMC:-"FETCH_SIZE" "WRITE_SIZE"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$OUT/pmc$i" -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variant --no-side > "$OUT/pmc$i.log" 2>&1
  st=$?; echo "pmc pass $i ($set) exit $st"; [ $st -eq 0 ] || exit $st
done
find "$OUT" -name "*.csv" | head -50
