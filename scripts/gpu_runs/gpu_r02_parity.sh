# parity suite + per-fixture report + error-ratio statistics + A/B vs a variant lib
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; st=$?; tail -6 gpurun_out/pytest_gpu.log; [ $st -le 1 ] || exit $st
timeout -k 10 300 python -u scripts/parity_report.py gpurun_out/r02_parity_report.json > gpurun_out/parity.log 2>&1 && grep -E "model/|torch" gpurun_out/parity.log &&
timeout -k 10 600 python -u scripts/parity_stats.py 16 > gpurun_out/parity_stats.log 2>&1 && cat gpurun_out/parity_stats.log &&
timeout -k 10 300 python -u scripts/ab_kernels.py ${AB_LIBS:-dstd-gcn_amd/libdstd_gcn_r01.so dstd-gcn_amd/libdstd_gcn.so} --rounds 5 > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log
