#!/bin/bash
# Round 6: assembly flash-attention dK/dV kernel — correctness, then A/B vs the HIP kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_fa
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fa_asm_gpu.py > $OUT/asm_tests.log 2>&1
rc=$?; tail -25 $OUT/asm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py > $OUT/attn_tests.log 2>&1
rc=$?; tail -3 $OUT/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for V in 0 1; do
  PIAMD_FA_ASM=$V timeout -k 10 200 python tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128;4,4096,16,128" > $OUT/bench_asm$V.log 2>&1 || { tail -20 $OUT/bench_asm$V.log; exit 1; }
  echo "== asm=$V"; cat $OUT/bench_asm$V.log
done
cd /tmp && for V in 0 1; do
  PIAMD_FA_ASM=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof$V -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/$OUT/prof$V.log 2>&1 || exit 1
done
