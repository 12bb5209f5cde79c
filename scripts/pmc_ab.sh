#!/bin/bash
# PMC counter passes over an A/B run of library variants (one pass per
# counter set, never combined with trace domains).  Stops at the first failure.
#   PMC_LIBS="a.so b.so" scripts/pmc_ab.sh   -> gpurun_out/${PROF_TAG:-pmcab}/pmc<i>
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/${PROF_TAG:-pmcab}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 2
LIBS=""
for l in ${PMC_LIBS:-libdstd_gcn.so}; do LIBS="$LIBS $REPO/dstd-gcn_amd/$l"; done
i=0
for set in ${PMC_SETS:-"SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$OUT/pmc$i" -o run -- python3 $REPO/scripts/ab_kernels.py $LIBS --rounds 1 --steps 2 > "$OUT/pmc$i.log" 2>&1
  st=$?; echo "pmc pass $i ($set) exit $st"; [ $st -eq 0 ] || exit $st
done
