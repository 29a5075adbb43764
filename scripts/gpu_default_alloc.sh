#!/bin/bash
# Default (framework allocator) GPU tier + smoke + bench + hipGraph decode bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gputest_def.log 2>&1
rc=$?
tail -6 gpurun_out/gputest_def.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_def.log 2>&1 || { tail -30 gpurun_out/smoke_def.log; exit 1; }
tail -1 gpurun_out/smoke_def.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_def.log 2>&1 || { tail -20 gpurun_out/bench_def.log; exit 1; }
tail -1 gpurun_out/bench_def.log | cut -c1-200; grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/bench_def.log
timeout -k 10 300 python tools/bench_generate.py --batch 1 8 --prompt 128 --gen 128 --modes graph > gpurun_out/gen_def.log 2>&1 || { tail -20 gpurun_out/gen_def.log; exit 1; }
grep "^{" gpurun_out/gen_def.log | cut -c1-200
