#!/bin/bash
# FA after the per-buffer LDS objects: attention GPU tests, then timing + kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128;4,4096,16,128;16,1024,32,64" > gpurun_out/fa_ab3.log 2>&1 || { tail -20 gpurun_out/fa_ab3.log; exit 1; }
grep "^{" gpurun_out/fa_ab3.log | cut -c1-230
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fa_prof4 -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/gpurun_out/fa_prof4.log 2>&1
