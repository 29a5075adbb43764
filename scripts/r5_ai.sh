#!/bin/bash
# Serving-batch FFN2 (K = 8192) A/B: packed GEMV slices + finalize (default) vs in-kernel atomic
# fixup vs the skinny MFMA GEMM; batch 8 / 32 hipGraph decode.
set -o pipefail
OUT=gpurun_out/r5_ai
mkdir -p $OUT
run() {
  timeout -k 10 400 env "$@" python3 tools/bench_generate.py --batch 8 32 --prompt 128 --gen 64 --modes graph > $OUT/gen.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen.log; exit 1; }
  echo "$@"; grep '^{' $OUT/gen.log | cut -c1-200
}
run PIAMD_X=0
run PIAMD_WO_FIXUP_MAX_M=64
run PIAMD_DENSE_MAX_K=8192
