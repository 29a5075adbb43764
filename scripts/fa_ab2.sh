#!/bin/bash
# FA A/B: attention GPU tests (default kernels), then bwd v1 vs v2 and fwd 4 vs 8 waves.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || exit $rc
S="96,1024,16,128;8,2048,16,128;4,4096,16,128"
for CFG in "1 4" "2 4" "2 8"; do
  set -- $CFG
  PIAMD_FA_BWD_V=$1 PIAMD_FA_FWD_WAVES=$2 timeout -k 10 200 python tools/bench_attn.py --no-sdpa --shapes "$S" > gpurun_out/fa_ab_$1_$2.log 2>&1 || { tail -20 gpurun_out/fa_ab_$1_$2.log; exit 1; }
  echo "== bwd v$1 fwd waves $2"; grep "^{" gpurun_out/fa_ab_$1_$2.log | cut -c1-220
done
cd /tmp && PIAMD_FA_FWD_WAVES=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fa_prof3 -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/gpurun_out/fa_prof3.log 2>&1
