#!/bin/bash
# Decode step anatomy: kernel trace of the single-launch (cooperative) batch-1 decode.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4d2_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_generate.py --batch 1 --prompt 128 --gen 32 --modes graph > $GRAFT_REPO_ROOT/gpurun_out/r4d2_trace.log 2>&1
echo "rocprof rc=$?"
tail -3 $GRAFT_REPO_ROOT/gpurun_out/r4d2_trace.log
ls -la $GRAFT_REPO_ROOT/gpurun_out/r4d2_trace/ 2>/dev/null | head
