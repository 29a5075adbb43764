#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/trace_aten_predictor.py > gpurun_out/r6x_trace.txt 2>&1 || { tail -20 gpurun_out/r6x_trace.txt; exit 1; }
grep -v "^/opt" gpurun_out/r6x_trace.txt | head -30 | cut -c1-200
