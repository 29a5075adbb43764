#!/bin/bash
# Full GPU tier (what the driver runs at round end) + smoke + the 1-GPU bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t3_tier.log 2>&1 || { tail -60 gpurun_out/r4t3_tier.log; exit 1; }
tail -3 gpurun_out/r4t3_tier.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r4t3_bench.log 2>&1 || { tail -20 gpurun_out/r4t3_bench.log; exit 1; }
grep "^{" gpurun_out/r4t3_bench.log | cut -c1-400
