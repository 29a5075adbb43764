#!/bin/bash
# rocprof kernel stats of the default bench step (HEAD), summary in gpurun_out/train_prof_stats.txt
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/train_prof -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/train_prof.log 2>&1 || { tail -20 gpurun_out/train_prof.log; exit 1; }
python3 tools/rocpd_stats.py $(find gpurun_out/train_prof -name "*.db" | head -1) --top 30 > gpurun_out/train_prof_stats.txt 2>&1
rm -rf gpurun_out/train_prof
tail -1 gpurun_out/train_prof.log | cut -c1-200
head -40 gpurun_out/train_prof_stats.txt
