#!/bin/bash
# Decode serving: generation bench (graph mode) + rocprofv3 kernel stats of batch-1 decode.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-head}
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_generate.py --batch 1 8 --prompt 128 --gen 128 --modes graph int8 > gpurun_out/gen_$TAG.log 2>&1 || { tail -20 gpurun_out/gen_$TAG.log; exit 1; }
grep "^{" gpurun_out/gen_$TAG.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_$TAG -o run -- python tools/bench_generate.py --batch 1 --prompt 128 --gen 64 --modes graph > gpurun_out/dprof_$TAG.log 2>&1 || { tail -20 gpurun_out/dprof_$TAG.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/dprof_$TAG/run_results.db --top 14 --tail 3000 > gpurun_out/dprof_$TAG.txt
cut -c1-150 gpurun_out/dprof_$TAG.txt
