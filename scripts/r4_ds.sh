#!/bin/bash
# Stored-dS flash-attention backward: numerics vs the recomputing dQ kernel and the fp32 reference,
# then fwd+bwd throughput with the dS scratch on / off, and a kernel trace of the bench shape.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_ds_gpu.py tests/test_attention_gpu.py > gpurun_out/r4_ds_tests.log 2>&1 || { tail -40 gpurun_out/r4_ds_tests.log; exit 1; }
tail -2 gpurun_out/r4_ds_tests.log
S="96,1024,16,128;8,2048,16,128;4,4096,16,128;16,1024,32,64"
for MB in 0 8192; do
  echo "== PIAMD_FA_DS_MAX_MB=$MB"
  PIAMD_FA_DS_MAX_MB=$MB timeout -k 10 300 python tools/bench_attn.py --no-sdpa --shapes "$S" > gpurun_out/r4_ds_bench_$MB.log 2>&1 || { tail -20 gpurun_out/r4_ds_bench_$MB.log; exit 1; }
  grep "^{" gpurun_out/r4_ds_bench_$MB.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_ds_prof -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $GRAFT_REPO_ROOT/gpurun_out/r4_ds_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4_ds_prof > gpurun_out/r4_ds_prof.txt 2>&1
head -12 gpurun_out/r4_ds_prof.txt
