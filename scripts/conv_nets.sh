#!/bin/bash
# Conv nets on 1 MI355X: ResNet-50 / MobileNetV2 training throughput (eager + hipGraph) and the
# kernel stats of a ResNet-50 and a MobileNetV2 step (no MIOpen kernel expected).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in resnet50 mobilenet_v2; do
  for G in "" "--graph"; do
    timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 $G > gpurun_out/cn_${M}${G}.log 2>&1 || { tail -20 gpurun_out/cn_${M}${G}.log; exit 1; }
    grep "^{" gpurun_out/cn_${M}${G}.log | cut -c1-300
  done
done
cd /tmp
for M in resnet50 mobilenet_v2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cn_prof_$M -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model $M --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/cn_prof_$M.log 2>&1 || exit 1
done
