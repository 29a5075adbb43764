#!/bin/bash
# ResNet-50 training step kernel trace (batch 128, bf16 autocast, channels_last).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_prof_rn50b -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model resnet50 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4_prof_rn50b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
grep "^{" gpurun_out/r4_prof_rn50b.log | cut -c1-200
