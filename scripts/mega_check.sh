#!/bin/bash
# Single-launch decode: numerics vs the per-op path, then batch-1 decode timing (mega vs per-op).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_decode_mega_gpu.py > gpurun_out/mega_test.log 2>&1
rc=$?; tail -15 gpurun_out/mega_test.log; [ $rc -eq 0 ] || exit $rc
PIAMD_DECODE_MEGA=1 timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/mega_bench.log 2>&1 || { tail -20 gpurun_out/mega_bench.log; exit 1; }
PIAMD_DECODE_MEGA=0 timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph >> gpurun_out/mega_bench.log 2>&1 || { tail -20 gpurun_out/mega_bench.log; exit 1; }
grep decode gpurun_out/mega_bench.log
