#!/bin/bash
# round 6 (r06e): the whole GPU suite on the tree with the per-sample block
# kernel (default schedule), the fp64 PReLU-slope partials and the
# calibrated 3x gradient bar; the gradient-bar calibration again (the native
# step's ratios after the fp64 slope); then the default bench line (with the
# per-leg CPU baselines) as the driver runs it
cd "$(dirname "$0")/../.." || exit 2
O=$PWD/gpurun_out/r06e
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
st=$?; tail -3 $O/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python -u scripts/grad_bar_calibration.py $O/grad_bar_calibration.json > $O/grad_bar.txt 2>&1 || exit 1
tail -4 $O/grad_bar.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06e/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["avg_launch_us"])
for k in ("variant_t75", "cmu_b256", "3dpw_b256"):
    print(k, d[k]["value"], d[k]["ms_per_step"], "cpu", d[k]["cpu_baseline"]["value"], "x", d[k]["vs_cpu"])
print("exact", d["exact_fp32"]["value"], "b32", d["eval_b32"]["ms_per_step"], "train", d["train_b32"]["ms_per_step"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["thread_sweep_seq_s"], "vs_cpu", d["vs_cpu"])
PY
