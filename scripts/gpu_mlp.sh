#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_agemm_gpu.py > gpurun_out/t_agemm.log 2>&1 || { echo tests-failed; tail -30 gpurun_out/t_agemm.log; exit 1; }
tail -2 gpurun_out/t_agemm.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_mlp.log 2>&1 || { echo e2e-failed; tail -20 gpurun_out/bench_mlp.log; exit 1; }
tail -1 gpurun_out/bench_mlp.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_mlp.log 2>&1 || { tail -30 gpurun_out/prof_mlp.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/prof_mlp/run_results.db --top 40 > gpurun_out/prof_mlp.txt
head -24 gpurun_out/prof_mlp.txt | cut -c1-150
