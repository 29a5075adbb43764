#!/bin/bash
# BERT-Large fp16 Predictor: residual-free post-LN and the few-row LayerNorm threshold A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for rm in 64 512; do
  PIAMD_LN_ROW_MAX=$rm timeout -k 10 240 python tools/bench_bert_infer.py --predictor-only --batches 1,128 --iters 30 \
    > gpurun_out/r6_bert_$rm.log 2>&1 || { tail -20 gpurun_out/r6_bert_$rm.log; exit 1; }
  echo "row_max=$rm"; grep '^{"model' gpurun_out/r6_bert_$rm.log
done
