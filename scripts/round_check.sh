set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
for dt in fp16 bf16; do
timeout -k 10 300 python tools/bench_bert_infer.py --dtype $dt --batches 1,128 --iters 20 --predictor-only 2>&1 | grep "^{" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert_fp16 -o run -- python tools/bench_bert_infer.py --dtype fp16 --batches 128 --iters 5 --predictor-only > gpurun_out/prof_bert_fp16.log 2>&1 || { tail -30 gpurun_out/prof_bert_fp16.log; exit 1; }
echo done
