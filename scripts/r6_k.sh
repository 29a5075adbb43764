#!/bin/bash
# Deferred LayerNorm (BERT post-LN at few rows): GPU tests + BERT-Large fp16 A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ln_defer_gpu.py tests/test_ln_fold_gpu.py > gpurun_out/r6k_tests.log 2>&1 || { tail -40 gpurun_out/r6k_tests.log; exit 1; }
tail -3 gpurun_out/r6k_tests.log
for d in 1 0; do
  PIAMD_LN_DEFER=$d timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,8,128 --iters 30 --predictor-only > gpurun_out/r6k_bert_$d.log 2>&1 || { tail -20 gpurun_out/r6k_bert_$d.log; exit 1; }
  echo "LN_DEFER=$d"; grep '^{' gpurun_out/r6k_bert_$d.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_prof -o run -- python tools/bench_bert_infer.py --dtype fp16 --batches 1 --iters 30 --predictor-only > gpurun_out/r6k_prof.log 2>&1 || { tail -30 gpurun_out/r6k_prof.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/r6k_prof/run_results.db --top 20 --tail 1200 > gpurun_out/r6k_prof.txt
head -30 gpurun_out/r6k_prof.txt | cut -c1-140
