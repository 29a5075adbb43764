#!/bin/bash
# BERT-Large fp16 Predictor with the B-deep skinny GEMM configs + skinny GEMM GPU tests.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_own_gpu.py tests/test_ln_fold_gpu.py > gpurun_out/r6_sgtest.log 2>&1 || { tail -30 gpurun_out/r6_sgtest.log; exit 1; }
tail -2 gpurun_out/r6_sgtest.log
timeout -k 10 240 python tools/bench_bert_infer.py --predictor-only --batches 1,128 --iters 30 > gpurun_out/r6_bert_b.log 2>&1 || { tail -20 gpurun_out/r6_bert_b.log; exit 1; }
grep '^{"model' gpurun_out/r6_bert_b.log
