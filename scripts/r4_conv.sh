#!/bin/bash
# Wide-head attention backward on own GEMMs + own 1x1-conv backward GEMMs: tests, conv-net
# throughput, and a MobileNetV2 kernel trace (no Cijk_* expected).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_gpu.py tests/test_conv_any_gpu.py > gpurun_out/r4_conv_tests.log 2>&1 || { tail -30 gpurun_out/r4_conv_tests.log; exit 1; }
tail -2 gpurun_out/r4_conv_tests.log
for M in resnet50 mobilenet_v2; do
  timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4_cn_$M.log 2>&1 || { tail -20 gpurun_out/r4_cn_$M.log; exit 1; }
  grep "^{" gpurun_out/r4_cn_$M.log | cut -c1-200
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_cn_prof_mbv2 -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model mobilenet_v2 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4_cn_prof_mbv2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4_cn_prof_mbv2 > gpurun_out/r4_cn_prof_mbv2.txt 2>&1
head -24 gpurun_out/r4_cn_prof_mbv2.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_decode_mega_gpu.py tests/test_infer_kernels_gpu.py > gpurun_out/r4_mega_tests.log 2>&1 || { tail -30 gpurun_out/r4_mega_tests.log; exit 1; }
tail -2 gpurun_out/r4_mega_tests.log
timeout -k 10 300 python -u tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/r4_gen_b1.log 2>&1 || { tail -20 gpurun_out/r4_gen_b1.log; exit 1; }
grep '^{' gpurun_out/r4_gen_b1.log
