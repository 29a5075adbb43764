#!/bin/bash
# Full GPU tier + a short headline bench (round-4 checkpoint).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_tier.log 2>&1 || { tail -40 gpurun_out/r4_tier.log; exit 1; }
tail -3 gpurun_out/r4_tier.log
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 > gpurun_out/r4_bench.log 2>&1 || { tail -20 gpurun_out/r4_bench.log; exit 1; }
grep '^{' gpurun_out/r4_bench.log
