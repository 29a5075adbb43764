#!/bin/bash
# Main-loop slot-schedule sweep of the assembly GEMM (wall, random bf16, three NT training shapes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_sched
mkdir -p $OUT
for S in "98304 2048 2048" "98304 2048 8192" "98304 8192 2048"; do
  set -- $S
  for V in v0 v8 v9 v10 v11 v12 v13 v0; do
    PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_s_$V.hsaco timeout -k 10 120 python3 tools/gemm_ab_probe.py --M $1 --N $2 --K $3 --impls asm --iters 20 --rounds 5 > $OUT/w.tmp 2>&1 || { echo "$V failed"; tail -3 $OUT/w.tmp; exit 1; }
    echo "$V $(grep '^{' $OUT/w.tmp)" | tee -a $OUT/sweep.txt
  done
done
