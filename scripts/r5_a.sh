#!/bin/bash
# New GPU tests of this round (fp32 split GEMMs, native graph fixes, program ops) + the GEMM PMC A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py tests/test_native_infer_gpu.py > gpurun_out/r5a_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r5a_tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
bash scripts/r5_pmc_ab.sh
