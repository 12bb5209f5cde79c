#!/bin/bash
# Build the aggregation microbenchmark against the in-tree library (CPU side).
cd "$(dirname "$0")" || exit 2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 agg_micro.cpp -o agg_micro \
  -L../../dstd-gcn_amd -ldstd_gcn -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 skinny_micro.cpp -o skinny_micro \
  -L../../dstd-gcn_amd -ldstd_gcn -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd'
# the same benchmark against variant libraries: MICRO_VARIANTS="nostream csg2 ..."
# builds skinny_micro_<name> linked with libdstd_gcn_<name>.so
for v in ${MICRO_VARIANTS:-}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 skinny_micro.cpp -o skinny_micro_$v \
    -L../../dstd-gcn_amd -l:libdstd_gcn_$v.so -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd' || exit 1
done
