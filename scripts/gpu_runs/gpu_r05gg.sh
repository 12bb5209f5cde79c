#!/bin/bash
# round 5 (r05gg): spatial backward aggregation with 32 / 64 channels per
# workgroup (k_aggc_bwd MF = 2 / 4: D read once per chunk, 2 / 1 dD partials
# instead of 4): gradients of one step compared, B=32 training A/B (3
# rounds), kernel trace of each
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05gg
mkdir -p $O
export TMPDIR=/tmp
for v in base cw32 cw64; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = base ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/grad_ab.py $O/g_$v.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python3 scripts/grad_ab.py --compare $O/g_base.npz $O/g_cw32.npz && python3 scripts/grad_ab.py --compare $O/g_base.npz $O/g_cw64.npz || exit 1
for r in 1 2 3; do
  for v in base cw32 cw64; do
    lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = base ] && lib=dstd-gcn_amd/libdstd_gcn.so
    DSTD_LIB=$R/$lib timeout -k 10 200 python -u scripts/train_ab.py 32 $v 2>&1 | grep -v amdgpu.ids >> $O/train_b32.txt || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05gg/train_b32.txt"):
    if " {" in l:
        t, j = l.split(" ", 1)
        d = json.loads(j)
        print(t, "B=32 ms", d["ms_per_step"], "host_issue_us", d["host_issue_us_per_step"])
PY
for v in base cw32 cw64; do
  lib=dstd-gcn_amd/libdstd_gcn_$v.so; [ $v = base ] && lib=dstd-gcn_amd/libdstd_gcn.so
  DSTD_LIB=$R/$lib timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tt_$v -o run -- python3 scripts/bench_train.py --batch 32 --steps 6 --warmup 3 > $O/tt_$v.log 2>&1 || exit 1
  python3 scripts/trace_summary.py $O/tt_$v/run_kernel_trace.csv 3 30 --marker k_prep_nctv --last 3 > $O/train_trace_summary_$v.txt || exit 1
  echo "== $v"; head -2 $O/train_trace_summary_$v.txt | tail -1; grep -E "k_aggc_bwd|k_adj_bwd_part" $O/train_trace_summary_$v.txt; tail -2 $O/train_trace_summary_$v.txt
done
