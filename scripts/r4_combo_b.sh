#!/bin/bash
# Round-4 verification batch, part B: conv-net throughput, cooperative decode tests + b1 decode,
# native fused_multi_transformer decode latency, MobileNetV2 / attention / decode kernel traces.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 600 python tools/bench_native_fmt.py --layers 4 --steps 64 > gpurun_out/r4c_native_fmt_bench.log 2>&1 || { tail -20 gpurun_out/r4c_native_fmt_bench.log; exit 1; }
grep "^{" gpurun_out/r4c_native_fmt_bench.log
for P in 0 1; do PIAMD_LN_BWD_PAIR=$P timeout -k 10 120 python tools/bench_ln_bwd.py || exit 1; done
for M in resnet50 mobilenet_v2; do
  timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4c_cn_$M.log 2>&1 || { tail -20 gpurun_out/r4c_cn_$M.log; exit 1; }
  grep "^{" gpurun_out/r4c_cn_$M.log | cut -c1-220
done
timeout -k 10 300 $T tests/test_decode_mega_gpu.py tests/test_infer_kernels_gpu.py > gpurun_out/r4c_mega_tests.log 2>&1 || { tail -30 gpurun_out/r4c_mega_tests.log; exit 1; }
tail -1 gpurun_out/r4c_mega_tests.log
timeout -k 10 300 python -u tools/bench_generate.py --batch 1 --prompt 128 --gen 128 --modes graph > gpurun_out/r4c_gen_b1.log 2>&1 || { tail -20 gpurun_out/r4c_gen_b1.log; exit 1; }
grep '^{' gpurun_out/r4c_gen_b1.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_mbv2 -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model mobilenet_v2 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_mbv2.log 2>&1 || exit 1
for MB in 0 8192; do
  PIAMD_FA_PERSIST=0 PIAMD_FA_DS_MAX_MB=$MB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_attn_$MB -o run -- python $GRAFT_REPO_ROOT/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;16,1024,32,64" > $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_attn_$MB.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4c_prof_mbv2 > gpurun_out/r4c_prof_mbv2.txt 2>&1
python tools/prof_summary.py gpurun_out/r4c_prof_attn_0 > gpurun_out/r4c_prof_attn_0.txt 2>&1
python tools/prof_summary.py gpurun_out/r4c_prof_attn_8192 > gpurun_out/r4c_prof_attn_8192.txt 2>&1
head -14 gpurun_out/r4c_prof_mbv2.txt
head -12 gpurun_out/r4c_prof_attn_0.txt
head -12 gpurun_out/r4c_prof_attn_8192.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_gen -o run -- python $GRAFT_REPO_ROOT/tools/bench_generate.py --batch 1 --prompt 128 --gen 64 --modes graph > $GRAFT_REPO_ROOT/gpurun_out/r4c_prof_gen.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4c_prof_gen > gpurun_out/r4c_prof_gen.txt 2>&1
head -16 gpurun_out/r4c_prof_gen.txt
