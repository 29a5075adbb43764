set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for v in base new; do
  if [ $v = base ]; then export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_base.so; else unset PIAMD_KERNEL_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/act2_$v -o run -- python tools/bench_bias_act.py > gpurun_out/act2_prof_$v.log 2>&1
  python tools/rocpd_stats.py gpurun_out/act2_$v/run_results.db --top 3 > gpurun_out/act2_stats_$v.txt 2>&1
  echo "== $v"; grep -h "^{" gpurun_out/act2_prof_$v.log; cut -c1-150 gpurun_out/act2_stats_$v.txt
done
unset PIAMD_KERNEL_LIB
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_new2.log 2>&1
tail -1 gpurun_out/bench_new2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/train_prof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/train_prof.log 2>&1
python tools/rocpd_stats.py gpurun_out/train_prof/run_results.db --top 40 > gpurun_out/train_stats.txt 2>&1
head -20 gpurun_out/train_stats.txt | cut -c1-150
rm -rf gpurun_out/train_prof gpurun_out/act2_base gpurun_out/act2_new
