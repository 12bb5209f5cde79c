#!/bin/bash
# round 5 (r05w): upper bound of a faster MFMA path in the streaming GEMM of
# the training step: the B=32 step with k_conv_stream's MFMAs ablated
# (csabl: -DDSTD_CS_ABL=1, wrong results, timing only) against the real one
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05w
mkdir -p $O
for r in 1 2; do
  for v in csabl new; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = new ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05w/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"])
PY
