#!/bin/bash
# Kernel trace of the batch-32 GPT-1.3B hipGraph decode (what limits the weight stream at M = 32).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_c
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/bench_generate.py --batch 32 --prompt 128 --gen 16 --modes graph > $OUT/gen32.log 2>&1 || { echo "prof failed"; tail -20 $OUT/gen32.log; exit 1; }
grep "^{" $OUT/gen32.log | cut -c1-300
python3 tools/prof_summary.py $OUT/prof > $OUT/summary.txt 2>&1; head -40 $OUT/summary.txt
