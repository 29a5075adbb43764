#!/bin/bash
# loop-efficiency probe of the assembly GEMM (default + ablated builds) and a kernel trace of the
# bench step on it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/agemm_check.py --stage probe --rounds 3 > gpurun_out/probe_default.log 2>&1 || { echo probe-failed; tail -5 gpurun_out/probe_default.log; exit 1; }
grep case gpurun_out/probe_default.log
for v in nodma noreads nomfma nobar; do
  PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_abl_$v.hsaco timeout -k 10 200 python -u tools/agemm_check.py --stage probe --rounds 3 > gpurun_out/probe_$v.log 2>&1 || { echo probe-$v-failed; tail -5 gpurun_out/probe_$v.log; exit 1; }
  grep case gpurun_out/probe_$v.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_asm -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_asm.log 2>&1 || { tail -30 gpurun_out/prof_asm.log; exit 1; }
python tools/rocpd_stats.py gpurun_out/prof_asm/run_results.db --top 40 > gpurun_out/prof_asm.txt
head -32 gpurun_out/prof_asm.txt | cut -c1-150
