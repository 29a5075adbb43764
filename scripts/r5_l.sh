#!/bin/bash
# BERT-Large fp16 Predictor: which kernels run INSIDE a run (tail of the trace = the last ~10 runs
# of the timed loop) vs model setup (weight uploads / casts), at batch 1 and 128.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_l
mkdir -p $OUT
for B in 1 128; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/p$B -o run -- python3 tools/bench_bert_infer.py --batches $B --iters 30 --dtype fp16 --predictor-only > $OUT/b$B.log 2>&1 || { echo "prof b$B failed"; tail -20 $OUT/b$B.log; exit 1; }
  grep '^{' $OUT/b$B.log | cut -c1-300
  DB=$(ls $OUT/p$B/*/*results.db $OUT/p$B/*results.db 2>/dev/null | head -1)
  python3 tools/rocpd_stats.py $DB --top 14 --tail 1700 > $OUT/stats_b$B.txt 2>&1
  cat $OUT/stats_b$B.txt | cut -c1-150
done
