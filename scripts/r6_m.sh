#!/bin/bash
# Column-sum reduce + tuned decode-shape skinny configs: GPU tests, decode A/B (dense FFN2 at K = 8192), GPT bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_colsum_gpu.py tests/test_groupnorm_gpu.py tests/test_agemm_gpu.py tests/test_gemm_own_gpu.py tests/test_ln_fold_gpu.py tests/test_ln_defer_gpu.py tests/test_infer_kernels_gpu.py tests/test_gemm_gpu.py > gpurun_out/r6m_tests.log 2>&1 || { tail -40 gpurun_out/r6m_tests.log; exit 1; }
tail -2 gpurun_out/r6m_tests.log
for k in 2048 8192; do
  PIAMD_DENSE_MAX_K=$k timeout -k 10 300 python tools/bench_generate.py --batch 8 32 --prompt 128 --gen 64 --modes graph > gpurun_out/r6m_dec_$k.log 2>&1 || { tail -20 gpurun_out/r6m_dec_$k.log; exit 1; }
  echo "DENSE_MAX_K=$k"; grep '^{' gpurun_out/r6m_dec_$k.log
done
timeout -k 10 300 python bench.py > gpurun_out/r6m_bench.log 2>&1 || { tail -30 gpurun_out/r6m_bench.log; exit 1; }
grep '^{' gpurun_out/r6m_bench.log
