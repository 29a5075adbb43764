#!/bin/bash
# Native predictor on the framework kernels: GPU tests + BERT-Large latency vs the Python Predictor
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_fast_gpu.py tests/test_native_infer_gpu.py > gpurun_out/r4_native_tests.log 2>&1 || { tail -40 gpurun_out/r4_native_tests.log; exit 1; }
grep -c PASSED gpurun_out/r4_native_tests.log
timeout -k 10 600 python -u tools/bench_native_bert.py --batches 1,32,128 > gpurun_out/r4_native_bert.jsonl 2>&1 || { tail -30 gpurun_out/r4_native_bert.jsonl; exit 1; }
grep '^{' gpurun_out/r4_native_bert.jsonl
