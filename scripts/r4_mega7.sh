#!/bin/bash
# Loader-wave decode kernel: attention-split sweep.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for NS in 16 4; do
  echo "== nsplit $NS"
  PIAMD_MEGA_NSPLIT=$NS timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m7_trace_$NS.log 2>&1 || { tail -20 gpurun_out/r4m7_trace_$NS.log; exit 1; }
  grep "^{" gpurun_out/r4m7_trace_$NS.log
done
