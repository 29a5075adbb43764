#!/bin/bash
# FA forward: persistent grid size A/B (workgroups per CU), kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_g
mkdir -p $OUT
cd /tmp
for w in 2 1 2 1; do
  PIAMD_FA_FWD_WGS=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/w$w -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $OUT/w$w.log 2>&1 || { echo "w$w failed"; exit 1; }
  python $GRAFT_REPO_ROOT/tools/rocpd_stats.py $OUT/w$w/run_results.db | grep -E 'fa_fwd' | sed "s/^/wgs=$w /"
done
