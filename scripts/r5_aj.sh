#!/bin/bash
# Decode attention split A/B at serving batches (single-pass 192-key workgroups vs 64 / 128-key splits).
set -o pipefail
OUT=gpurun_out/r5_aj
mkdir -p $OUT
run() {
  timeout -k 10 400 env "$@" python3 tools/bench_generate.py --batch 8 32 --prompt 128 --gen 64 --modes graph > $OUT/gen.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen.log; exit 1; }
  echo "$@"; grep '^{' $OUT/gen.log | cut -c1-200
}
run PIAMD_DECODE_CHUNK=0
run PIAMD_DECODE_CHUNK=64
run PIAMD_DECODE_CHUNK=128
run PIAMD_DECODE_CHUNK=32
