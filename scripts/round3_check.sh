#!/bin/bash
# Round-3 HEAD check: full GPU tier, smoke, driver-style bench, conv nets.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gputest_r3.log 2>&1
rc=$?; tail -4 gpurun_out/gputest_r3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3.log 2>&1 || { tail -30 gpurun_out/smoke_r3.log; exit 1; }
tail -1 gpurun_out/smoke_r3.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r3.log 2>&1 || { tail -20 gpurun_out/bench_r3.log; exit 1; }
tail -1 gpurun_out/bench_r3.log | cut -c1-300
bash scripts/conv_nets.sh
