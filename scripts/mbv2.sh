#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "conv or depthwise or group" > gpurun_out/mb_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mb_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_resnet.py --model mobilenet_v2 --steps 10 > gpurun_out/mb_e.log 2>&1 || { tail -10 gpurun_out/mb_e.log; exit 1; }
grep "^{" gpurun_out/mb_e.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/mb_prof -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model mobilenet_v2 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/mb_prof.log 2>&1
