set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
for dt in fp16 bf16; do
timeout -k 10 300 python tools/bench_bert_infer.py --dtype $dt --batches 1,32,128 --iters 20 --predictor-only 2>&1 | grep "^{" || exit 1
done | tee gpurun_out/bert_r2.jsonl
