#!/bin/bash
# FA backward dK/dV kernel: correctness (attention GPU tests on the default = pipelined kernel),
# then old (PIAMD_FA_BWD_V=1) vs new timing at the bench shape, and a kernel-trace of both.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || exit $rc
for V in 1 2; do
  PIAMD_FA_BWD_V=$V timeout -k 10 200 python tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128;4,4096,16,128;16,1024,32,64" > gpurun_out/fa_ab_v$V.log 2>&1 || { tail -20 gpurun_out/fa_ab_v$V.log; exit 1; }
  echo "== v$V"; cat gpurun_out/fa_ab_v$V.log
done
cd /tmp && for V in 1 2; do
  PIAMD_FA_BWD_V=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fa_prof_v$V -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/gpurun_out/fa_prof_v$V.log 2>&1 || exit 1
done
