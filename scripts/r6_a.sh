#!/bin/bash
# Round-6 HEAD check: full GPU tier (no -x), smoke, bench.py.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_a
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?
tail -25 $OUT/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
