#!/bin/bash
# Round-4 verification batch: stored-dS attention backward, wide-head own-GEMM backward, dense fp32
# split conv + own 1x1 conv backward, conv-net throughput + MobileNetV2 trace, cooperative decode.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 500 $T tests/test_attention_ds_gpu.py tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py > gpurun_out/r4c_attn_tests.log 2>&1 || { tail -40 gpurun_out/r4c_attn_tests.log; exit 1; }
tail -1 gpurun_out/r4c_attn_tests.log
timeout -k 10 400 $T -s tests/test_native_fmt_gpu.py tests/test_native_fast_gpu.py > gpurun_out/r4c_native_tests.log 2>&1 || { tail -40 gpurun_out/r4c_native_tests.log; exit 1; }
grep -E "decode step|run_ms|passed|failed" gpurun_out/r4c_native_tests.log | tail -8
timeout -k 10 500 $T tests/test_conv_any_gpu.py tests/test_conv_gpu.py tests/test_conv_bwd_gpu.py > gpurun_out/r4c_conv_tests.log 2>&1 || { tail -40 gpurun_out/r4c_conv_tests.log; exit 1; }
tail -1 gpurun_out/r4c_conv_tests.log
timeout -k 10 300 $T tests/test_kernels_gpu.py tests/test_norm_gpu.py tests/test_op_cases_gpu.py > gpurun_out/r4c_ln_tests.log 2>&1 || { tail -40 gpurun_out/r4c_ln_tests.log; exit 1; }
tail -1 gpurun_out/r4c_ln_tests.log
for P in 0 1; do PIAMD_LN_BWD_PAIR=$P timeout -k 10 120 python tools/bench_ln_bwd.py; done
S="96,1024,16,128;8,2048,16,128;4,4096,16,128;16,1024,32,64"
for CFG in "0 0" "8192 0" "8192 1"; do
  set -- $CFG
  echo "== PIAMD_FA_DS_MAX_MB=$1 PIAMD_FA_PERSIST=$2"
  PIAMD_FA_DS_MAX_MB=$1 PIAMD_FA_PERSIST=$2 timeout -k 10 300 python tools/bench_attn.py --no-sdpa --shapes "$S" > gpurun_out/r4c_attn_bench_$1_$2.log 2>&1 || { tail -20 gpurun_out/r4c_attn_bench_$1_$2.log; exit 1; }
  grep "^{" gpurun_out/r4c_attn_bench_$1_$2.log | cut -c1-220
done
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r4c_bench.log 2>&1 || { tail -20 gpurun_out/r4c_bench.log; exit 1; }
grep "^{" gpurun_out/r4c_bench.log | cut -c1-400
