#!/bin/bash
# Build the aggregation microbenchmark against the in-tree library (CPU side).
cd "$(dirname "$0")" || exit 2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 agg_micro.cpp -o agg_micro \
  -L../../dstd-gcn_amd -ldstd_gcn -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 skinny_micro.cpp -o skinny_micro \
  -L../../dstd-gcn_amd -ldstd_gcn -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd'
# the same benchmark against a variant library (e.g. libdstd_gcn_nostream.so)
if [ -f ../../dstd-gcn_amd/libdstd_gcn_nostream.so ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 skinny_micro.cpp -o skinny_micro_nostream \
    -L../../dstd-gcn_amd -l:libdstd_gcn_nostream.so -Wl,-rpath,'$ORIGIN/../../dstd-gcn_amd'
fi
