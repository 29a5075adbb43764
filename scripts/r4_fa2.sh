#!/bin/bash
# Stored-dS backward with deferred stores + diagonal persistent forward: tests and A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 500 $T tests/test_attention_ds_gpu.py tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py > gpurun_out/r4f_attn_tests.log 2>&1 || { tail -40 gpurun_out/r4f_attn_tests.log; exit 1; }
tail -1 gpurun_out/r4f_attn_tests.log
S="96,1024,16,128;8,2048,16,128;4,4096,16,128;16,1024,32,64"
for CFG in "0 0" "8192 0" "0 1" "8192 1"; do
  set -- $CFG
  echo "== PIAMD_FA_DS_MAX_MB=$1 PIAMD_FA_PERSIST=$2"
  PIAMD_FA_DS_MAX_MB=$1 PIAMD_FA_PERSIST=$2 timeout -k 10 300 python tools/bench_attn.py --no-sdpa --shapes "$S" > gpurun_out/r4f_attn_bench_$1_$2.log 2>&1 || { tail -20 gpurun_out/r4f_attn_bench_$1_$2.log; exit 1; }
  grep "^{" gpurun_out/r4f_attn_bench_$1_$2.log | cut -c1-220
done
cd /tmp
PIAMD_FA_PERSIST=1 PIAMD_FA_DS_MAX_MB=8192 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4f_prof_attn -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;16,1024,32,64" > $GRAFT_REPO_ROOT/gpurun_out/r4f_prof_attn.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4f_prof_attn > gpurun_out/r4f_prof_attn.txt 2>&1
head -12 gpurun_out/r4f_prof_attn.txt
