#!/bin/bash
# Batch-32 hipGraph decode (GPT-3 1.3B, prompt 128): per-kernel census of the decode steps (trace tail).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_ag${SUFFIX}
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace -d $OUT/p -o run -- python3 tools/bench_generate.py --batch 32 --prompt 128 --gen 64 --modes graph > $OUT/gen.log 2>&1 || { echo "prof failed"; tail -20 $OUT/gen.log; exit 1; }
grep '^{' $OUT/gen.log | cut -c1-300
DB=$(ls $OUT/p/*/*results.db $OUT/p/*results.db 2>/dev/null | head -1)
python3 tools/rocpd_stats.py $DB --top 25 --tail 3000 > $OUT/stats.txt 2>&1
cut -c1-150 $OUT/stats.txt
