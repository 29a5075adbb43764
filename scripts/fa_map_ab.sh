#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PIAMD_FA_BWD_MAP=1 timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests_map.log 2>&1
rc=$?; tail -2 gpurun_out/fa_tests_map.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && for M in 0 1; do
  PIAMD_FA_BWD_MAP=$M timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fa_map$M -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128" > $GRAFT_REPO_ROOT/gpurun_out/fa_map$M.log 2>&1 || exit 1
  grep "^{" $GRAFT_REPO_ROOT/gpurun_out/fa_map$M.log | cut -c1-200
done
