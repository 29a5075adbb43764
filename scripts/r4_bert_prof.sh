#!/bin/bash
# BERT-Large fp16 Predictor (BASELINE config 4) on the own GEMMs: exact-GELU epilogue test, latency at
# batch 1 / 32 / 128, copy-kernel sources, and a kernel trace at batch 1 and 128 (zero Cijk_* expected).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_own_gpu.py -k "exact_gelu or small_gemm or gemm_nt or fused_epi" > gpurun_out/r4_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r4_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r4_gemm_tests.log
timeout -k 10 400 python tools/bench_bert_infer.py --dtype fp16 --batches 1,32,128 --iters 30 --predictor-only > gpurun_out/r4_bert_fp16.log 2>&1 || { tail -30 gpurun_out/r4_bert_fp16.log; exit 1; }
grep "^{" gpurun_out/r4_bert_fp16.log
timeout -k 10 300 python tools/trace_copies.py --layers 2 --batch 128 > gpurun_out/r4_trace_copies.txt 2>&1 || { tail -30 gpurun_out/r4_trace_copies.txt; exit 1; }
head -20 gpurun_out/r4_trace_copies.txt
for b in 1 128; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_bert_b$b -o run -- python tools/bench_bert_infer.py --dtype fp16 --batches $b --iters 5 --predictor-only > gpurun_out/r4_prof_bert_b$b.log 2>&1 || { tail -30 gpurun_out/r4_prof_bert_b$b.log; exit 1; }
done
python tools/prof_summary.py gpurun_out/r4_prof_bert_b1 > gpurun_out/r4_prof_bert_b1.txt 2>&1
python tools/prof_summary.py gpurun_out/r4_prof_bert_b128 > gpurun_out/r4_prof_bert_b128.txt 2>&1
head -30 gpurun_out/r4_prof_bert_b1.txt
head -30 gpurun_out/r4_prof_bert_b128.txt
