#!/bin/bash
# Round 6: viterbi + native graph LRU GPU tests, then assembly dK/dV ablation timings.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_viterbi_gpu.py tests/test_native_infer_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r6_fa_abl.sh
