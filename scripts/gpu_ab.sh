# GPU parity suite (fail-fast) + A/B of library variants: AB_LIBS="a.so b.so"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; st=$?; tail -8 gpurun_out/pytest_gpu.log; [ $st -le 1 ] || exit $st
for c in ${AB_CONFIGS:-h36m}; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $AB_LIBS --rounds 5 --config $c > gpurun_out/ab_$c.log 2>&1; st=$?; echo "== $c"; cat gpurun_out/ab_$c.log; [ $st -eq 0 ] || exit $st
done
