set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_norm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/normtest.log 2>&1 || { tail -40 gpurun_out/normtest.log; exit 1; }
tail -2 gpurun_out/normtest.log
for cfg in "--rows 65536 --hidden 2048" "--rows 65536 --hidden 2048 --dtype fp16" "--rows 16384 --hidden 5120" "--rows 16384 --hidden 5120 --rms --dropout 0" "--rows 8192 --hidden 8192" "--rows 4096 --hidden 16384 --dtype fp16"; do
  timeout -k 10 120 python tools/bench_ln.py $cfg --iters 30 || exit 1
done | tee gpurun_out/ln_bench.jsonl
timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | tail -1
