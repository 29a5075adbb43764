#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_dwconv.py > gpurun_out/r4dw.log 2>&1 || { tail -20 gpurun_out/r4dw.log; exit 1; }
grep "^{" gpurun_out/r4dw.log
