#!/bin/bash
# BERT-Large fp16: LayerNorm deferral up to 512 rows (batch 2 / 4) vs the 128-row default.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 128 512; do
  PIAMD_LN_DEFER_MAX_M=$m timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,2,4 --iters 30 --predictor-only > gpurun_out/r6n_bert_$m.log 2>&1 || { tail -20 gpurun_out/r6n_bert_$m.log; exit 1; }
  echo "DEFER_MAX_M=$m"; grep '^{"model' gpurun_out/r6n_bert_$m.log
done
