#!/bin/bash
# rocprof kernel stats of the BERT-Large fp16 Predictor at batch 1 (hipGraph replays)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/bert_prof -o run -- python3 tools/bench_bert_infer.py --batches 1 --predictor-only --iters 50 > gpurun_out/bert_prof.log 2>&1 || { tail -20 gpurun_out/bert_prof.log; exit 1; }
python3 tools/rocpd_stats.py $(find gpurun_out/bert_prof -name "*.db" | head -1) --top 25 --tail 3000 > gpurun_out/bert_prof_stats.txt 2>&1
tail -45 gpurun_out/bert_prof_stats.txt
