#!/bin/bash
# aggregation microbenchmark (+ optional PMC pass) on the GPU box
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/agg
# AGG_CASES: FORM:AC pairs (DSTD_AGG_FORM, DSTD_AGG_AC)
for fc in ${AGG_CASES:-0:0}; do
  form=${fc%%:*}; ac=${fc##*:}
  echo "DSTD_AGG_FORM=$form DSTD_AGG_AC=$ac" >> gpurun_out/agg/micro.txt
  DSTD_AGG_FORM=$form DSTD_AGG_AC=$ac timeout -k 10 120 scripts/micro/agg_micro ${AGG_ARGS:-64 64} >> gpurun_out/agg/micro.txt 2>&1
  st=$?; [ $st -eq 0 ] || { cat gpurun_out/agg/micro.txt; exit $st; }
done
cat gpurun_out/agg/micro.txt
if [ -n "${AGG_PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  i=0
  for set in $AGG_PMC; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/agg/pmc$i" -o run -- "$GRAFT_REPO_ROOT/scripts/micro/agg_micro" ${AGG_ARGS:-64 64} > "$GRAFT_REPO_ROOT/gpurun_out/agg/pmc$i.log" 2>&1
    echo "pmc $i exit $?"
  done
fi
