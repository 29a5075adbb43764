#!/bin/bash
# Two-rows-per-wave LayerNorm forward for narrow rows: norm tests, LN microbench, BERT-Large fp16 Predictor A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_af
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_norm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r2 in 1 0; do
  PIAMD_LN_ROWS2=$r2 timeout -k 10 120 python3 tools/bench_ln.py --rows 16384 --hidden 1024 --dtype fp16 --dropout 0 > $OUT/ln_$r2.log 2>&1 || { tail -20 $OUT/ln_$r2.log; exit 1; }
  echo "rows2=$r2 $(grep '^{' $OUT/ln_$r2.log)"
done
for r2 in 1 0; do
  PIAMD_LN_ROWS2=$r2 timeout -k 10 400 python3 tools/bench_bert_infer.py --predictor-only --batch 128 > $OUT/bert_$r2.log 2>&1 || { tail -20 $OUT/bert_$r2.log; exit 1; }
  echo "rows2=$r2 $(grep '^{' $OUT/bert_$r2.log | tail -1 | cut -c1-200)"
done
