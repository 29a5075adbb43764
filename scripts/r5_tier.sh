#!/bin/bash
# Full GPU tier (what the driver runs at round end) + smoke + the 1-GPU bench + ResNet ATen census.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_tier
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/tier.log 2>&1 || { tail -60 $OUT/tier.log; exit 1; }
tail -3 $OUT/tier.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep "^{" $OUT/bench.log | cut -c1-400
timeout -k 10 300 python3 tools/trace_aten_step.py > $OUT/aten_rn50.txt 2>&1 || { echo "aten trace failed"; tail -20 $OUT/aten_rn50.txt; exit 1; }
head -8 $OUT/aten_rn50.txt
