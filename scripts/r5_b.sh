#!/bin/bash
# (1) global_load_lds DMA variant of the assembly GEMM: correctness (every layout / epilogue) +
# wall A/B on three NT shapes; (2) where the BERT-Large fp16 Predictor's device copies come from.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_b
mkdir -p $OUT
PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_s_g10.hsaco timeout -k 10 300 python3 tools/agemm_check.py --stage small > $OUT/g0_small.log 2>&1 || { echo "g0 small failed"; tail -20 $OUT/g0_small.log; exit 1; }
tail -3 $OUT/g0_small.log
for S in "98304 2048 2048" "98304 2048 8192" "98304 8192 2048"; do
  set -- $S
  for V in v0 g0 v10 g10 v0; do
    PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_s_$V.hsaco timeout -k 10 120 python3 tools/gemm_ab_probe.py --M $1 --N $2 --K $3 --impls asm --iters 20 --rounds 5 > $OUT/w.tmp 2>&1 || { echo "$V failed"; tail -3 $OUT/w.tmp; exit 1; }
    echo "$V $(grep '^{' $OUT/w.tmp)" | tee -a $OUT/sweep.txt
  done
done
timeout -k 10 300 python3 tools/trace_copies.py --batch 1 --layers 4 > $OUT/copies_b1.txt 2>&1 || { echo "trace b1 failed"; tail -20 $OUT/copies_b1.txt; }
timeout -k 10 300 python3 tools/trace_copies.py --batch 128 --layers 4 > $OUT/copies_b128.txt 2>&1 || { echo "trace b128 failed"; tail -20 $OUT/copies_b128.txt; }
tail -40 $OUT/copies_b1.txt
