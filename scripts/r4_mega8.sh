#!/bin/bash
# Loader-wave decode kernel with fp16 attention partials and a 16-wide combine: tests + split sweep.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_decode_mega_gpu.py > gpurun_out/r4m8_tests.log 2>&1 || { tail -30 gpurun_out/r4m8_tests.log; exit 1; }
tail -1 gpurun_out/r4m8_tests.log
for NS in 8 16; do
  PIAMD_MEGA_NSPLIT=$NS timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m8_trace_$NS.log 2>&1 || { tail -20 gpurun_out/r4m8_trace_$NS.log; exit 1; }
  echo "nsplit $NS $(grep '^{' gpurun_out/r4m8_trace_$NS.log | head -1)"
  grep '"attn"\|"out"' gpurun_out/r4m8_trace_$NS.log
  PIAMD_MEGA_NSPLIT=$NS timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/r4m8_gen_$NS.log 2>&1 || { tail -20 gpurun_out/r4m8_gen_$NS.log; exit 1; }
  grep "^{" gpurun_out/r4m8_gen_$NS.log | cut -c1-200
done
