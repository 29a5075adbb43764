#!/bin/bash
# Single-launch decode at long context: attention splits 8 (default) vs 16, batch 1, prompt 1024 / 128.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for ns in 8 16; do
  for p in 1024 128; do
    PIAMD_MEGA_NSPLIT=$ns timeout -k 10 200 python tools/bench_generate.py --batch 1 --prompt $p --gen 128 --modes graph > gpurun_out/r6p_${ns}_$p.log 2>&1 || { tail -20 gpurun_out/r6p_${ns}_$p.log; exit 1; }
    echo "NSPLIT=$ns prompt=$p"; grep '^{' gpurun_out/r6p_${ns}_$p.log
  done
done
