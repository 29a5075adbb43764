#!/bin/bash
# Flash-attention A/B: FA GPU tests on the new build, then rocprofv3 kernel stats of the base build
# (PIAMD_KERNEL_LIB) and the new one at the GPT-3 1.3B training shape.
# usage: scripts/fa_ab.sh [SHAPES]   (default "64,1024,16,128")
set -o pipefail
export TMPDIR=/tmp
SHAPES=${1:-"64,1024,16,128"}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or attention" > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
for v in base new; do
  if [ $v = base ]; then export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_base.so; else unset PIAMD_KERNEL_LIB; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/fa_$v -o run -- python tools/bench_attn.py --no-sdpa --shapes "$SHAPES" > gpurun_out/fa_bench_$v.log 2>&1 || { tail -20 gpurun_out/fa_bench_$v.log; exit 1; }
  python tools/rocpd_stats.py gpurun_out/fa_$v/run_results.db --top 6 > gpurun_out/fa_stats_$v.txt
  echo "== $v"; grep -h "fa_\|{" gpurun_out/fa_bench_$v.log gpurun_out/fa_stats_$v.txt | cut -c1-200
done
