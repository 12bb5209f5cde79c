#!/bin/bash
# round 4 (r04c; r04d = the same minus the parity / training suites, which
# passed at r04c on unchanged sources, with the distributed tests last): forward -- VALU trims of the split GC kernels, 12-wave fused
# temporal at H36M, slot-ordered phase-1/3 tables, late spatial residual:
# parity suite, same-box A/B against the round-3 library (r03), the 8-wave
# fused kernel (tf8) and 3-wave spatial (sp3), phase timeline.  Training --
# batched tanh-outer kernels, LDS-staged BN merge, weight-gradient stream:
# the training suite (incl. the bit-identity test of the two streams) and the
# training-step A/B main / nows (one stream) / r03.  Kernel trace of the bench.
cd "$(dirname "$0")/../.." || exit 2
R="$PWD"
O=$R/gpurun_out/r04d
mkdir -p $O
L=dstd-gcn_amd
export DSTD_AB_FOREIGN_LIB=1
for cfg in h36m cmu 3dpw; do
  echo "# $cfg" >> $O/ab.txt
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn_r03.so $L/libdstd_gcn_tf8.so $L/libdstd_gcn.so $L/libdstd_gcn_sp3.so --config $cfg --rounds 5 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt | cut -c1-400
for r in 1 2; do
  for lib in libdstd_gcn libdstd_gcn_nows libdstd_gcn_r03; do
    DSTD_LIB="$R/$L/$lib.so" timeout -k 10 300 python -u scripts/bench_train.py --batch 32 256 > $O/train_$lib.$r.log 2>&1
    st=$?; echo "$lib round $r exit $st"; grep metric $O/train_$lib.$r.log | cut -c1-420; [ $st -eq 0 ] || exit $st
  done
done
timeout -k 10 120 python -u scripts/timeline.py $L/libdstd_gcn_stamps.so --hl > $O/timeline.txt 2>&1; st=$?
grep -v amdgpu.ids $O/timeline.txt | head -60; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
unset DSTD_AB_FOREIGN_LIB
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-variant --no-side > "$O/kt.log" 2>&1)
st=$?; echo "kt exit $st"; [ $st -eq 0 ] || exit $st
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 13 24
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1
st=$?; tail -3 $O/pytest_dist.log; [ $st -eq 0 ] || exit $st
