#!/bin/bash
# tanh epilogue of the skinny GEMM: tests (incl. LN fold / defer / skinny GEMM suites) + BERT fp16.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_small_gemm_tanh_gpu.py tests/test_ln_defer_gpu.py tests/test_ln_fold_gpu.py tests/test_gemm_own_gpu.py tests/test_native_fast_gpu.py > gpurun_out/r6y_tests.log 2>&1 || { tail -40 gpurun_out/r6y_tests.log; exit 1; }
tail -2 gpurun_out/r6y_tests.log
timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,128 --iters 30 --predictor-only > gpurun_out/r6y_bert.log 2>&1 || { tail -20 gpurun_out/r6y_bert.log; exit 1; }
grep '^{"model' gpurun_out/r6y_bert.log
