#!/bin/bash
# Decode mega kernel, loader-wave variant as default: GPU tests + latency at two prompt lengths.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_decode_mega_gpu.py tests/test_infer_kernels_gpu.py > gpurun_out/r4m6_tests.log 2>&1 || { tail -30 gpurun_out/r4m6_tests.log; exit 1; }
tail -1 gpurun_out/r4m6_tests.log
timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m6_trace.log 2>&1 || { tail -20 gpurun_out/r4m6_trace.log; exit 1; }
grep "^{" gpurun_out/r4m6_trace.log
for P in 128 1024; do
timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt $P --gen 128 --modes graph > gpurun_out/r4m6_gen_p$P.log 2>&1 || { tail -20 gpurun_out/r4m6_gen_p$P.log; exit 1; }
grep "^{" gpurun_out/r4m6_gen_p$P.log | cut -c1-300
done
