#!/bin/bash
# New GPU tests (embedding lookup, GroupNorm, LN deferral) + long-context split A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_embedding_lookup_gpu.py tests/test_groupnorm_gpu.py tests/test_ln_defer_gpu.py tests/test_kernels_gpu.py > gpurun_out/r6q_tests.log 2>&1 || { tail -40 gpurun_out/r6q_tests.log; exit 1; }
tail -2 gpurun_out/r6q_tests.log
bash scripts/r6_p.sh
