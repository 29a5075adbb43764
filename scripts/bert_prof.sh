set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in fp16 bf16; do
timeout -k 10 300 python tools/bench_bert_infer.py --dtype $dt --batches 128 --iters 20 --predictor-only 2>&1 | grep "^{" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert_$dt -o run -- python tools/bench_bert_infer.py --dtype $dt --batches 128 --iters 5 --predictor-only > gpurun_out/prof_bert_$dt.log 2>&1 || { tail -30 gpurun_out/prof_bert_$dt.log; exit 1; }
done
