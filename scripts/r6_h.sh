#!/bin/bash
# FA forward 8-wave kernel: correctness, then 4- vs 8-wave kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fa_asm_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for w in 8 4 8 4; do
  PIAMD_FA_FWD_NW=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/w$w -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $OUT/w$w.log 2>&1 || { echo "w$w failed"; exit 1; }
  python $GRAFT_REPO_ROOT/tools/rocpd_stats.py $OUT/w$w/run_results.db | grep -E 'fa_fwd' | sed "s/^/nw=$w /"
done
