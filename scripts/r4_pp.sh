#!/bin/bash
# 8-wave ping-pong NT GEMM: correctness (small shapes, then the GEMM test files), then the GPT
# training-shape bench against hipBLASLt with and without the ping-pong kernel.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
PIAMD_AGEMM_PP=1 timeout -k 10 120 python -u tools/agemm_check.py --stage small > gpurun_out/r4_pp_small.log 2>&1 || { tail -30 gpurun_out/r4_pp_small.log; exit 1; }
tail -3 gpurun_out/r4_pp_small.log
PIAMD_AGEMM_PP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_agemm_gpu.py tests/test_gemm_own_gpu.py > gpurun_out/r4_pp_tests.log 2>&1 || { tail -30 gpurun_out/r4_pp_tests.log; exit 1; }
tail -2 gpurun_out/r4_pp_tests.log
PIAMD_AGEMM_PP=1 timeout -k 10 300 python -u tools/agemm_check.py --stage bench --rounds 5 > gpurun_out/r4_pp_bench.jsonl 2>&1 || { tail -30 gpurun_out/r4_pp_bench.jsonl; exit 1; }
timeout -k 10 300 python -u tools/agemm_check.py --stage bench --rounds 5 > gpurun_out/r4_nopp_bench.jsonl 2>&1 || { tail -30 gpurun_out/r4_nopp_bench.jsonl; exit 1; }
grep -h '"fwd"\|"dgrad"' gpurun_out/r4_pp_bench.jsonl gpurun_out/r4_nopp_bench.jsonl | grep -v hipblaslt
grep -h hipblaslt gpurun_out/r4_pp_bench.jsonl | grep -v wgrad
PIAMD_AGEMM_PP=1 timeout -k 10 200 python -u tools/agemm_check.py --stage bench --rounds 5 --T 16384 --shapes bqkv,bout,bffn1,bffn2 > gpurun_out/r4_pp_bert.jsonl 2>&1 || { tail -30 gpurun_out/r4_pp_bert.jsonl; exit 1; }
grep -v wgrad gpurun_out/r4_pp_bert.jsonl
