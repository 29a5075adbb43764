#!/bin/bash
# End-of-round HEAD check: full GPU tier, smoke, driver-style bench, single-launch decode bench + trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gputest_final.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_final.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -30 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-200
PIAMD_DECODE_MEGA=1 timeout -k 10 300 python tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/mega_bench_final.log 2>&1 || { tail -20 gpurun_out/mega_bench_final.log; exit 1; }
grep decode gpurun_out/mega_bench_final.log
timeout -k 10 300 python tools/mega_trace.py > gpurun_out/mega_trace_final.log 2>&1 || { tail -20 gpurun_out/mega_trace_final.log; exit 1; }
grep -v Warn gpurun_out/mega_trace_final.log | tail -6
