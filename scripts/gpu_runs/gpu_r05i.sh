#!/bin/bash
# round 5 (r05i): training -- float4 BatchNorm applies (libdstd_gcn.so)
# against the scalar loops (libdstd_gcn_bnscalar.so, -DDSTD_BN_NOVEC): the
# training suite, then two interleaved rounds of bench.train_leg at B=32 / 256
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fast.py > $O/pytest_train.log 2>&1
st=$?; tail -1 $O/pytest_train.log; [ $st -eq 0 ] || exit $st
for r in 1 2; do
  for v in bnscalar:dstd-gcn_amd/libdstd_gcn_bnscalar.so new:dstd-gcn_amd/libdstd_gcn.so; do
    for B in 32 256; do
      DSTD_LIB=$R/${v#*:} timeout -k 10 200 python -u scripts/train_ab.py $B ${v%%:*} >> $O/train_ab.txt 2>&1
      st=$?; [ $st -eq 0 ] || { tail -5 $O/train_ab.txt; exit $st; }
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05i/train_ab.txt"):
    if " {" not in l:
        continue
    tag, js = l.split(" ", 1)
    d = json.loads(js)
    print(tag, d["workload"].split(",")[2].split(":")[0], "ms", d["ms_per_step"], "host_issue_us", d.get("host_issue_us_per_step"),
          "graph ms", d["graph_replay"]["ms_per_step"])
PY
