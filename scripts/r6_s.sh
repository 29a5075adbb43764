#!/bin/bash
# Decode mega GPU tests (split switch) + decode at prompt 128 / 1024 with the default + ResNet ATen trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_mega_gpu.py > gpurun_out/r6s_tests.log 2>&1 || { tail -40 gpurun_out/r6s_tests.log; exit 1; }
tail -2 gpurun_out/r6s_tests.log
for p in 1024 128; do
  timeout -k 10 200 python tools/bench_generate.py --batch 1 --prompt $p --gen 128 --modes graph > gpurun_out/r6s_dec_$p.log 2>&1 || { tail -20 gpurun_out/r6s_dec_$p.log; exit 1; }
  echo "prompt=$p"; grep '^{' gpurun_out/r6s_dec_$p.log
done
bash scripts/r6_r.sh
