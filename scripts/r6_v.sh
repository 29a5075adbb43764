#!/bin/bash
# BERT-Large fp16 Predictor at HEAD: batch 1 / 2 / 128 + batch-1 census.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,2,128 --iters 30 --predictor-only > gpurun_out/r6v_bert.log 2>&1 || { tail -20 gpurun_out/r6v_bert.log; exit 1; }
grep '^{"model' gpurun_out/r6v_bert.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6v_prof -o run -- python tools/bench_bert_infer.py --dtype fp16 --batches 1 --iters 30 --predictor-only > gpurun_out/r6v_prof.log 2>&1 || { tail -30 gpurun_out/r6v_prof.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/r6v_prof/run_results.db --top 12 --tail 1200 > gpurun_out/r6v_prof.txt
rm -rf gpurun_out/r6v_prof
tail -14 gpurun_out/r6v_prof.txt | cut -c1-140
