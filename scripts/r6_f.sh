#!/bin/bash
# FA forward schedule sweep (DMA spacing) by kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_f
mkdir -p $OUT
cd /tmp
for n in fwdgap1 fwdgap2 fwdgap1 fwdgap2; do
  PIAMD_FA_HSACO=$GRAFT_REPO_ROOT/paddle_infer_amd/_lib/abl/fa_$n.hsaco timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $OUT/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python $GRAFT_REPO_ROOT/tools/rocpd_stats.py $OUT/$n/run_results.db | grep -E 'fa_fwd|dkdv|fa_dq' | sed "s/^/$n /"
done
