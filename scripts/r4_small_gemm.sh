#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_own_gpu.py -k "small or gemm_nt or linear" > gpurun_out/r4_sg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_sg_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/tune_small_gemm.py --dtype fp16 --iters 20 > gpurun_out/r4_sg_tune.jsonl 2> gpurun_out/r4_sg_tune.err
rc=$?; cat gpurun_out/r4_sg_tune.jsonl | cut -c1-400; exit $rc
