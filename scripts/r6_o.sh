#!/bin/bash
# Training-step census at HEAD (column-sum reduce), BERT deferral threshold A/B, decode batch 16.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/train_prof.sh || exit 1
bash scripts/r6_n.sh || exit 1
timeout -k 10 300 python tools/bench_generate.py --batch 16 --prompt 128 --gen 64 --modes graph > gpurun_out/r6o_dec16.log 2>&1 || { tail -20 gpurun_out/r6o_dec16.log; exit 1; }
grep '^{' gpurun_out/r6o_dec16.log
