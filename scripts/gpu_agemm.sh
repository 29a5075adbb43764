#!/bin/bash
# assembly GEMM bring-up: correctness, per-shape timing vs hipBLASLt, end-to-end bench both ways
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/agemm_check.py --stage small > gpurun_out/agemm_small.log 2>&1 || { echo small-failed; tail -5 gpurun_out/agemm_small.log; exit 1; }
grep -v '"ok": true' gpurun_out/agemm_small.log | tail -5
timeout -k 10 400 python -u tools/agemm_check.py --stage bench --rounds 3 > gpurun_out/agemm_bench.log 2>&1 || { echo bench-failed; tail -5 gpurun_out/agemm_bench.log; exit 1; }
grep shape gpurun_out/agemm_bench.log | python -c "import sys,json; [print(d['shape'],d['pass'],d['impl'],d['ms'],d['tflops'],d['vs_blaslt'],d['max_diff_vs_blaslt']) for d in map(json.loads,sys.stdin)]"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_asm.log 2>&1 || { echo e2e-asm-failed; tail -5 gpurun_out/bench_asm.log; exit 1; }
tail -1 gpurun_out/bench_asm.log
PIAMD_GEMM=blas timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_blas.log 2>&1 || { echo e2e-blas-failed; exit 1; }
tail -1 gpurun_out/bench_blas.log
