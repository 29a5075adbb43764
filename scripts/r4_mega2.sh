#!/bin/bash
# Decode mega kernel: attention-split sweep after the parallel-load partial combine.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $T tests/test_decode_mega_gpu.py > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -1 gpurun_out/r4m_tests.log
for NS in 4 8 16; do
  echo "== trace nsplit $NS"
  PIAMD_MEGA_NSPLIT=$NS timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m_trace_$NS.log 2>&1 || { tail -20 gpurun_out/r4m_trace_$NS.log; exit 1; }
  grep "^{" gpurun_out/r4m_trace_$NS.log
done
for NS in 1 4 8; do
  echo "== generate nsplit $NS"
  PIAMD_MEGA_NSPLIT=$NS timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/r4m_gen_$NS.log 2>&1 || { tail -20 gpurun_out/r4m_gen_$NS.log; exit 1; }
  grep "^{" gpurun_out/r4m_gen_$NS.log | cut -c1-300
done
