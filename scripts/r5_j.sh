#!/bin/bash
# Templated single-launch decode step: GPT-1.3B (both variants), GPT-350M width, GQA 4:1 + rotary
# against the per-op path; then the batch-1 generate bench (regression check of the 1.3B kernel).
set -o pipefail
OUT=gpurun_out/r5_j
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_decode_mega_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/tests.log | tail -20
timeout -k 10 300 python3 tools/bench_generate.py --batch 1 --prompt 128 --gen 64 --modes graph int8 > $OUT/gen1.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen1.log; exit 1; }
grep '^{' $OUT/gen1.log
