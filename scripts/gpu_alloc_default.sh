#!/bin/bash
# Whole GPU tier + 1-GPU bench under the framework allocator (FLAGS_allocator_strategy=auto_growth).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FLAGS_allocator_strategy=auto_growth timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gputest_alloc.log 2>&1
rc=$?
tail -12 gpurun_out/gputest_alloc.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
FLAGS_allocator_strategy=auto_growth timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_alloc.log 2>&1 || { tail -20 gpurun_out/bench_alloc.log; exit 1; }
echo "== auto_growth"; tail -1 gpurun_out/bench_alloc.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_caching.log 2>&1 || { tail -20 gpurun_out/bench_caching.log; exit 1; }
echo "== caching"; tail -1 gpurun_out/bench_caching.log | cut -c1-400
