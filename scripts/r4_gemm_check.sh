#!/bin/bash
# Round-4 own-GEMM check: new kernels' numerics, the existing asm tests, a short bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gemm_own_gpu.py tests/test_agemm_gpu.py tests/test_gemm_gpu.py > gpurun_out/r4_gemm_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4_gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r4_bench.log 2>&1
rc=$?
tail -3 gpurun_out/r4_bench.log
exit $rc
