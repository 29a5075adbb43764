#!/bin/bash
# A/B: bench with the assembly FA forward on / off (same box), then a census with it on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_i
for m in 7 3 7 3; do
  PIAMD_FA_ASM=$([ $m = 7 ] && echo 1 || echo bwd) timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r6_i/bench_$m.log 2>&1 || { tail -20 gpurun_out/r6_i/bench_$m.log; exit 1; }
  echo "asm_mask=$m $(tail -1 gpurun_out/r6_i/bench_$m.log | cut -c1-160)"
done
bash scripts/bench_prof.sh r6fwd > /dev/null 2>&1 || exit 1
head -22 gpurun_out/prof_r6fwd.txt | cut -c1-150
