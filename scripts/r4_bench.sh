#!/bin/bash
# Headline bench (driver contract) + a kernel-stats profile of the training step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r4b_bench.log 2>&1 || { tail -20 gpurun_out/r4b_bench.log; exit 1; }
grep "^{" gpurun_out/r4b_bench.log | cut -c1-600
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4b_prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r4b_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4b_prof > gpurun_out/r4b_prof.txt 2>&1
head -30 gpurun_out/r4b_prof.txt
