#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_fast_gpu.py -k large > gpurun_out/r4_native_tests2.log 2>&1 || { grep -n "AssertionError\|released\|run_ms\|error" gpurun_out/r4_native_tests2.log | head -20; exit 1; }
tail -2 gpurun_out/r4_native_tests2.log
