#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Stops at the first
# step that ends abnormally (fault / abort / timeout); plain test failures
# (pytest exit 1) still let the later steps run.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
ok_status() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
st=$?; echo "pytest exit $st"; tail -25 gpurun_out/pytest_gpu.log
ok_status $st || exit $st

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?; echo "smoke exit $st"; tail -3 gpurun_out/smoke.log
[ $st -eq 0 ] || ok_status $st || exit $st

if [ -n "${BENCH_ARGS+x}" ] || [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-seconds 5} > gpurun_out/bench.log 2>&1
  st=$?; echo "bench exit $st"; tail -5 gpurun_out/bench.log
fi
if [ -n "${DIST_BENCH:-}" ] && [ $st -eq 0 ]; then
  # the RCCL code path (broadcast, sharding, metric all_reduce) at one rank
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_dist1.log 2>&1
  st=$?; echo "dist bench exit $st"; tail -3 gpurun_out/bench_dist1.log
fi
exit $st
