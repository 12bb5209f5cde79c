#!/bin/bash
# Variant libraries for same-box A/B (scripts/ab_kernels.py): each NAME=DEFS
# pair builds dstd-gcn_amd/libdstd_gcn_NAME.so from the current sources.
#   scripts/build_variants.sh tf8=-DDSTD_TF_NW_H36M=8 sp3=-DDSTD_HL_WPE=3
cd "$(dirname "$0")/../dstd-gcn_amd" || exit 2
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  make -j8 VARIANT="$name" DEFS="$defs" > /dev/null 2>"/tmp/build_$name.err" || { cat "/tmp/build_$name.err"; exit 1; }
  echo "built libdstd_gcn_$name.so ($defs)"
done
