#!/bin/bash
# lookup_table_v2 on the own gather: inference / native / embedding GPU tests + BERT fp16.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_embedding_lookup_gpu.py tests/test_ln_defer_gpu.py tests/test_native_infer_gpu.py tests/test_native_fast_gpu.py $(ls tests/test_infer*_gpu.py tests/test_bert*_gpu.py 2>/dev/null) > gpurun_out/r6w_tests.log 2>&1 || { tail -40 gpurun_out/r6w_tests.log; exit 1; }
tail -2 gpurun_out/r6w_tests.log
timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,128 --iters 30 --predictor-only > gpurun_out/r6w_bert.log 2>&1 || { tail -20 gpurun_out/r6w_bert.log; exit 1; }
grep '^{"model' gpurun_out/r6w_bert.log
