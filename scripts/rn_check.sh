#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "norm or bn or batch or conv or resnet" > gpurun_out/rn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rn_tests.log; [ $rc -eq 0 ] || exit $rc
for M in resnet50 mobilenet_v2; do
  timeout -k 10 200 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/rn_$M.log 2>&1 || { tail -10 gpurun_out/rn_$M.log; exit 1; }
  grep "^{" gpurun_out/rn_$M.log | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/rn_prof -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/rn_prof.log 2>&1
