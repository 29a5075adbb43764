#!/bin/bash
# ResNet-50 training step kernel profile (HIP conv path). usage: scripts/resnet_prof.sh [TAG]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-resnet}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python tools/bench_resnet.py --mode hip --batch 128 --steps 3 > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/prof_$TAG/run_results.db --top 45 > gpurun_out/prof_$TAG.txt
head -50 gpurun_out/prof_$TAG.txt | cut -c1-150
