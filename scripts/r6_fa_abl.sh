#!/bin/bash
# Ablation builds of the assembly dK/dV kernel (numerically wrong; timing only): which part of the
# tile loop costs what. Kernel time from rocprofv3 --kernel-trace at the bench shape.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_abl
mkdir -p $OUT
cd /tmp
for n in ${ABL_LIST:-full nodma nobar novalu noreads nomfma}; do
  PIAMD_FA_HSACO=$GRAFT_REPO_ROOT/paddle_infer_amd/_lib/abl/fa_$n.hsaco timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  python $GRAFT_REPO_ROOT/tools/rocpd_stats.py $OUT/$n/run_results.db | grep -E 'dkdv|fa_dq|fa_fwd' | sed "s/^/$n /"
done
