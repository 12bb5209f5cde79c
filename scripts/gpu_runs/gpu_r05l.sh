#!/bin/bash
# round 5 (r05l): HIP runtime knobs against the launch-bound legs (B=32 eval
# eager / graph replay, B=32 training step eager / graphed) and the launch
# gaps of eager vs graph replay at B=32 (kernel traces)
cd "$(dirname "$0")/../.." || exit 2
R=$PWD
O=$R/gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
run() {  # label, then KNOB=VALUE ...
  local l=$1; shift
  env "$@" timeout -k 10 240 python -u scripts/env_knobs.py --label "$l" 2>&1 | grep -v amdgpu.ids >> $O/knobs.txt
}
run base || exit 1
run pcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run pcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run gq1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 || exit 1
run gq4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 || exit 1
run hdp0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 || exit 1
run devka0 HIP_FORCE_DEV_KERNARG=0 || exit 1
run gbs64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
run base2 || exit 1
cat $O/knobs.txt
for m in eager graph; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$m -o tr -- python3 scripts/env_knobs.py --trace $m > $O/tr_$m.log 2>&1 || exit 1
  f=$(find $O/tr_$m -name '*kernel_trace.csv' | head -1)
  python3 scripts/gap_summary.py "$f" 1400 > $O/gaps_$m.txt || exit 1
  head -20 $O/gaps_$m.txt
done
