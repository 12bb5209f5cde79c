#!/bin/bash
# round 6 (r06ak): SQ counters of the block kernel (issue / wait / VALU / MFMA /
# LDS) -- VERDICT r05 weak #2's reading of the dominant kernel, redone for
# k_block_fused; two separate --pmc passes of 8 SQ counters each
cd "$(dirname "$0")/../.." || exit 2
PROF_TAG=r06ak PMC_LIBS="libdstd_gcn.so" bash scripts/pmc_ab.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/r06ak > gpurun_out/r06ak/summary.txt
cat gpurun_out/r06ak/summary.txt
