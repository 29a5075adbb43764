set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_attention_varlen_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fatest.log 2>&1 || { tail -40 gpurun_out/fatest.log; exit 1; }
tail -2 gpurun_out/fatest.log
S="64,1024,16,128"
for extra in "" "--dtype fp16" "--dropout 0.1" "--mask 1" "--causal 0"; do
  timeout -k 10 120 python tools/bench_attn.py --shapes $S --no-sdpa $extra || exit 1
done | tee gpurun_out/fa_bench.jsonl
