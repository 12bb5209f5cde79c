#!/bin/bash
# PMC passes (one counter set per run) over a microbenchmark binary:
#   PMC_BIN=scripts/micro/x PMC_TAG=name PMC_SETS="A,B C,D" bash scripts/gpu_pmc_bin.sh
cd "$(dirname "$0")/.." || exit 2
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${PMC_TAG:-pmc}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- "$R/$PMC_BIN" > "$O/kt.log" 2>&1
echo "kt exit $?"
i=0
for set in $PMC_SETS; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$O/pmc$i" -o run -- "$R/$PMC_BIN" > "$O/pmc$i.log" 2>&1
  st=$?; echo "pmc $i exit $st"; [ $st -eq 0 ] || exit $st
done
