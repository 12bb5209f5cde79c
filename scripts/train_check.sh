#!/bin/bash
# GPU check of the training path: parity tests, training-step bench and a
# kernel-trace profile of the bench.  Output under gpurun_out/${TAG:-train}.
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/${TAG:-train}"
mkdir -p "$OUT"
cd "$REPO" || exit 2
timeout -k 10 900 python -m pytest tests/test_gpu_train.py -q -p no:cacheprovider > "$OUT/tests.log" 2>&1
st=$?; echo "tests exit $st"; tail -3 "$OUT/tests.log"; [ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python scripts/bench_train.py ${BENCH_ARGS:---batch 32 256} > "$OUT/bench.log" 2>&1
st=$?; echo "bench exit $st"; grep metric "$OUT/bench.log"; [ $st -eq 0 ] || exit $st
if [ -n "${PROFILE:-1}" ]; then
  export TMPDIR=/tmp
  cd /tmp || exit 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$REPO/scripts/bench_train.py" --batch 32 --steps 10 --warmup 3 > "$OUT/prof.log" 2>&1
  echo "profile exit $?"
fi
