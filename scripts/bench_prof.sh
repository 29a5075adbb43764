#!/bin/bash
# 1-GPU bench + rocprofv3 kernel stats of the bench step. usage: scripts/bench_prof.sh [TAG] [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-head}; shift
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 "$@" > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 2 "$@" > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/prof_$TAG/run_results.db --top 40 > gpurun_out/prof_$TAG.txt
head -30 gpurun_out/prof_$TAG.txt | cut -c1-150
