#!/bin/bash
# Per-kernel VGPR / spill / occupancy / LDS summary of a HIP source (gfx950).
# usage: scripts/kres.sh dstd-gcn_amd/csrc/dstd_adj.hip [extra hipcc flags]
src=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$src" -o /tmp/kres.o "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | awk '
  /Function Name/ {if (n) print line; n=$3; line=n; next}
  /^VGPRs:/ {line=line" vgpr="$2} /^AGPRs:/ {line=line" agpr="$2}
  /ScratchSize/ {line=line" scratch="$NF} /Occupancy/ {line=line" occ="$NF}
  /VGPRs Spill/ {line=line" vspill="$NF} /SGPRs Spill/ {line=line" sspill="$NF}
  /LDS Size/ {line=line" lds="$NF}
  END {print line}' | c++filt | sed 's/(dstd::[A-Za-z]*Args)//'
