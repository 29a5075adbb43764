set -e
export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_base.so; else unset PIAMD_KERNEL_LIB; fi
  echo "$v $(timeout -k 10 120 python tools/bench_ln.py --rows 32768 2>gpurun_out/ln_err_$v.log | tail -1)"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ln_$v -o run -- python tools/bench_ln.py --rows 32768 > gpurun_out/ln_prof_$v.log 2>&1
  python tools/rocpd_stats.py gpurun_out/ln_$v/run_results.db --top 6 > gpurun_out/ln_stats_$v.txt 2>&1 || find gpurun_out/ln_$v | head
  echo "== $v"; cut -c1-150 gpurun_out/ln_stats_$v.txt
done
