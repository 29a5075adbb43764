set -e
export TMPDIR=/tmp
python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_varlen_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or attention" > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -3 gpurun_out/fa_tests.log
for v in base new; do
  if [ $v = base ]; then export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_base.so; else unset PIAMD_KERNEL_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fa_$v -o run -- python tools/bench_attn.py --shapes "32,1024,16,128" > gpurun_out/fa_bench_$v.log 2>&1
  python tools/rocpd_stats.py gpurun_out/fa_$v/run_results.db --top 8 > gpurun_out/fa_stats_$v.txt
  echo "== $v"; grep "fa_\|{" gpurun_out/fa_bench_$v.log gpurun_out/fa_stats_$v.txt | cut -c1-170
done
