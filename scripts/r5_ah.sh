#!/bin/bash
# LayerNorm fold in the skinny GEMM: numerics tests, inference GPU tests, batch 8 / 32 decode A/B.
set -o pipefail
OUT=gpurun_out/r5_ah
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ln_fold_gpu.py tests/test_infer_kernels_gpu.py tests/test_decode_mega_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for f in 1 0; do
  PIAMD_LN_FOLD=$f timeout -k 10 400 python3 tools/bench_generate.py --batch 8 32 --prompt 128 --gen 64 --modes graph > $OUT/gen_$f.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen_$f.log; exit 1; }
  echo "fold=$f"; grep '^{' $OUT/gen_$f.log
done
