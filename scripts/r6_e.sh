#!/bin/bash
# FA forward change check: attention GPU tests, then bench_attn + kernel trace at the bench shape.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py tests/test_fa_asm_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128;4,4096,16,128" > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.log | grep shape
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py $OUT/prof/run_results.db | head -8
