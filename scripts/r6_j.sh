#!/bin/bash
# HEAD check after the container re-creation: 1-GPU bench + batch-32 decode LN-fold A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r6j_bench.log 2>&1 || { tail -30 gpurun_out/r6j_bench.log; exit 1; }
grep '^{' gpurun_out/r6j_bench.log
for f in 1 0; do
  PIAMD_LN_FOLD=$f timeout -k 10 200 python tools/bench_generate.py --batch 32 --prompt 128 --gen 64 --modes graph > gpurun_out/r6j_dec_$f.log 2>&1 || { tail -20 gpurun_out/r6j_dec_$f.log; exit 1; }
  echo "LN_FOLD=$f"; grep '^{' gpurun_out/r6j_dec_$f.log
done
timeout -k 10 240 python tools/bench_resnet.py --mode hip --batch 128 --steps 20 > gpurun_out/r6j_resnet.log 2>&1 || { tail -20 gpurun_out/r6j_resnet.log; exit 1; }
grep '^{' gpurun_out/r6j_resnet.log
bash scripts/resnet_prof.sh r6j_resnet
