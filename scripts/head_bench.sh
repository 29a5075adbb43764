#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/agemm_check.py --stage bench > gpurun_out/agemm_bench.log 2>&1 || { tail -20 gpurun_out/agemm_bench.log; exit 1; }
tail -25 gpurun_out/agemm_bench.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_head.log 2>&1 || { tail -20 gpurun_out/bench_head.log; exit 1; }
tail -1 gpurun_out/bench_head.log | cut -c1-300
