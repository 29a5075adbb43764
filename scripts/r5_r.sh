#!/bin/bash
# Mega decode, templated kernel with K/V rows staged together: tests + plain vs loader-wave kernel.
set -o pipefail
OUT=gpurun_out/r5_r
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_decode_mega_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for L in 0 1; do
  PIAMD_MEGA_LOADER=$L timeout -k 10 300 python3 tools/bench_generate.py --batch 1 --prompt 128 --gen 64 --modes graph > $OUT/gen_l$L.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen_l$L.log; exit 1; }
  echo "loader=$L $(grep '^{' $OUT/gen_l$L.log | cut -c1-200)"
done
PIAMD_MEGA_LOADER=0 timeout -k 10 300 python3 tools/bench_generate.py --model gpt3-350m --batch 1 --prompt 128 --gen 64 --modes graph > $OUT/gen_350m.log 2>&1 || { echo "gen350 failed"; tail -20 $OUT/gen_350m.log; exit 1; }
echo "350m $(grep '^{' $OUT/gen_350m.log | cut -c1-220)"
