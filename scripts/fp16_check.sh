set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_infer_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp16test.log 2>&1 || { tail -40 gpurun_out/fp16test.log; exit 1; }
tail -2 gpurun_out/fp16test.log
timeout -k 10 300 python tools/bench_bert_infer.py --dtype fp16 --batches 1,32,128 --iters 20 > gpurun_out/bert_fp16.jsonl 2>&1 || { tail -30 gpurun_out/bert_fp16.jsonl; exit 1; }
cat gpurun_out/bert_fp16.jsonl | grep -v Warn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python tools/bench_bert_infer.py --dtype fp16 --batches 128 --iters 5 > gpurun_out/prof_bert.log 2>&1 || { tail -30 gpurun_out/prof_bert.log; exit 1; }
find gpurun_out/prof_bert -name "*kernel_stats.csv" | head -3
