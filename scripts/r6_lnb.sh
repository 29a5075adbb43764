#!/bin/bash
# LN backward A/B at the GPT-1.3B training shape: base (previous build) vs residual-gradient prefetch.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for v in base new; do
  if [ $v = base ]; then export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_base.so; else unset PIAMD_KERNEL_LIB; fi
  echo "$v $(timeout -k 10 120 python tools/bench_ln_bwd.py 2>gpurun_out/lnb_err_$v.log | tail -1)" || exit 1
done
done
unset PIAMD_KERNEL_LIB
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_gpu.py tests/test_kernels_gpu.py > gpurun_out/r6_lntest.log 2>&1 || { tail -30 gpurun_out/r6_lntest.log; exit 1; }
tail -1 gpurun_out/r6_lntest.log
