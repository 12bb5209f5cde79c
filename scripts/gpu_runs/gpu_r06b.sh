#!/bin/bash
# round 6 (r06b): the per-sample block kernel (k_block_fused) -- parity suite
# (incl. test_block_fused_schedule_bit_identical), then same-box interleaved
# A/B of the forward at H36M / CMU / 3DPW B=256: new (fused blocks), nobf (the
# same tree with -DDSTD_NO_BFUSED: round 5's two launches per block), noprio
# (round 5's HEAD without the spatial younger-wave priority), r04 (round 4's
# library) -- VERDICT r05 items 1 and 5; then the bench's RCCL path at one
# rank (item 6)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1
st=$?; tail -3 $O/pytest_parity.log; [ $st -eq 0 ] || exit $st
export DSTD_AB_FOREIGN_LIB=1
L=$R/dstd-gcn_amd
for cfg in h36m cmu 3dpw; do
  timeout -k 10 400 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_nobf.so $L/libdstd_gcn_noprio.so \
    $L/libdstd_gcn_r04.so --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  echo $cfg; tail -4 $O/ab_$cfg.txt
done
unset DSTD_AB_FOREIGN_LIB
B="bench.py --gpus 1 --no-variant --no-side --no-cpu-baseline"
timeout -k 10 300 python -u $B > $O/plain_b256.json 2> $O/plain_b256.err || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 $B > $O/dist1_b256.json 2> $O/dist1_b256.err || exit 1
timeout -k 10 300 python -u $B --global-batch 2048 > $O/plain_g2048.json 2> $O/plain_g2048.err || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29532 $B --global-batch 2048 > $O/dist1_g2048.json 2> $O/dist1_g2048.err || exit 1
python3 - <<'PY'
import json
for n in ("plain_b256", "dist1_b256", "plain_g2048", "dist1_g2048"):
    d = json.loads(open(f"gpurun_out/r06b/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["scaling"], d["config"]["global_batch"], d["roofline"]["kernel"],
          d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
PY
