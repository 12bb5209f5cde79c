# torchrun N=1 vs plain N=1 (the bench's N=1 point under the driver's two launchers), 50 steps each
set -o pipefail
mkdir -p gpurun_out
A="--steps 50 --warmup 10 --no-cpu-baseline --no-variant"
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531"
for i in 1 2; do
  timeout -k 10 120 python bench.py $A 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.load(sys.stdin); print('plain', d['ms_per_step'], d['roofline']['avg_launch_us'])" &&
  timeout -k 10 180 $TR bench.py $A 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.load(sys.stdin); print('torchrun', d['ms_per_step'], d['roofline']['avg_launch_us'])" || exit 1
done
