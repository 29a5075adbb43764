#!/bin/bash
# Flash-attention dK/dV kernel with the next tile's DMA spread over the S/dP k-steps: correctness
# (attention GPU tests) + fwd/bwd timing at the GPT bench shape and S = 2048.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_e
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128;8,2048,16,128" > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof > $OUT/summary.txt 2>&1; head -12 $OUT/summary.txt
