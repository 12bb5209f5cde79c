#!/bin/bash
# round 6 (r06a): VERDICT r05 items 5 and 6.
#  (1) CMU B=256 same-box interleaved A/B: HEAD, HEAD without the spatial
#      younger-wave priority (DSTD_SETPRIO_SP=0), the round-4 library
#      (git archive cabdfc5, built in-tree); H36M the same for reference
#  (2) the bench's RCCL path at one rank (torch.distributed.run, nccl), weak
#      B=256 and strong --global-batch 2048, beside the plain N=1 lines
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r06a
mkdir -p $O
export DSTD_AB_FOREIGN_LIB=1
L=$R/dstd-gcn_amd
for cfg in cmu h36m; do
  timeout -k 10 300 python -u scripts/ab_kernels.py $L/libdstd_gcn.so $L/libdstd_gcn_noprio.so $L/libdstd_gcn_r04.so \
    --config $cfg --rounds 5 --steps 20 > $O/ab_$cfg.txt 2>&1 || exit 1
  tail -3 $O/ab_$cfg.txt
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
    d = json.loads(open(f"gpurun_out/r06a/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["scaling"], d["config"]["global_batch"])
PY
