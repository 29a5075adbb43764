#!/bin/bash
# Round-5 GEMM schedule adopted: finer DMA-gap sweep, GEMM GPU tests, the driver-style bench,
# a step profile, the batch-32 decode profile and the BERT copy trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_d
mkdir -p $OUT
for S in "98304 2048 2048" "98304 8192 2048"; do
  set -- $S
  for V in v10 v14 v15 v10; do
    PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_s_$V.hsaco timeout -k 10 120 python3 tools/gemm_ab_probe.py --M $1 --N $2 --K $3 --impls asm --iters 20 --rounds 5 > $OUT/w.tmp 2>&1 || { echo "$V failed"; tail -3 $OUT/w.tmp; exit 1; }
    echo "$V $(grep '^{' $OUT/w.tmp)" | tee -a $OUT/sweep.txt
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_agemm_gpu.py tests/test_gemm_own_gpu.py tests/test_gemm_f32_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
grep "^{" $OUT/bench.log | cut -c1-300
timeout -k 10 300 python3 tools/gemm_ab_probe.py --M 98304 --N 2048 --K 2048 --iters 20 --rounds 5 > $OUT/ab_out.jsonl 2>&1 && cat $OUT/ab_out.jsonl | grep "^{"
timeout -k 10 300 python3 tools/trace_copies.py --batch 1 --layers 2 > $OUT/copies_b1.txt 2>&1 || { echo "trace failed"; tail -20 $OUT/copies_b1.txt; }
head -50 $OUT/copies_b1.txt
bash scripts/r5_c.sh
