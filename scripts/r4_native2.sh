#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_fast_gpu.py -k large > gpurun_out/r4_native_tests2.log 2>&1 || { tail -12 gpurun_out/r4_native_tests2.log; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_native_fast_gpu.py tests/test_native_infer_gpu.py > gpurun_out/r4_native_tests.log 2>&1 || { tail -20 gpurun_out/r4_native_tests.log; exit 1; }
tail -2 gpurun_out/r4_native_tests.log
timeout -k 10 600 python -u tools/bench_native_bert.py --batches 1,32,128 > gpurun_out/r4_native_bert.jsonl 2>&1 || { tail -30 gpurun_out/r4_native_bert.jsonl; exit 1; }
grep '^{' gpurun_out/r4_native_bert.jsonl
