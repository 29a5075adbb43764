#!/bin/bash
# Decode mega kernel with a dedicated loader wave: numerics first, then phase timeline and latency.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
PIAMD_MEGA_LOADER=1 timeout -k 10 240 $T tests/test_decode_mega_gpu.py > gpurun_out/r4m5_tests.log 2>&1 || { tail -30 gpurun_out/r4m5_tests.log; exit 1; }
tail -1 gpurun_out/r4m5_tests.log
for LW in 1 0; do
  echo "== loader $LW"
  PIAMD_MEGA_LOADER=$LW timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m5_trace_$LW.log 2>&1 || { tail -20 gpurun_out/r4m5_trace_$LW.log; exit 1; }
  grep "^{" gpurun_out/r4m5_trace_$LW.log
  PIAMD_MEGA_LOADER=$LW timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/r4m5_gen_$LW.log 2>&1 || { tail -20 gpurun_out/r4m5_gen_$LW.log; exit 1; }
  grep "^{" gpurun_out/r4m5_gen_$LW.log | cut -c1-300
done
