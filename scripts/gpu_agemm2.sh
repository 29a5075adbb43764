#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/agemm_check.py --stage small > gpurun_out/agemm_small.log 2>&1 || { echo small-failed; grep -v '"ok": true' gpurun_out/agemm_small.log | tail -8; exit 1; }
tail -1 gpurun_out/agemm_small.log
timeout -k 10 200 python -u tools/agemm_check.py --stage probe --rounds 3 > gpurun_out/probe_default.log 2>&1 || { echo probe-failed; tail -5 gpurun_out/probe_default.log; exit 1; }
grep case gpurun_out/probe_default.log
PIAMD_AGEMM_HSACO=paddle_infer_amd/_lib/piamd_agemm_abl_nodma.hsaco timeout -k 10 200 python -u tools/agemm_check.py --stage probe --rounds 3 > gpurun_out/probe_nodma.log 2>&1 && grep case gpurun_out/probe_nodma.log
timeout -k 10 400 python -u tools/agemm_check.py --stage bench --rounds 3 > gpurun_out/agemm_bench.log 2>&1 || { echo bench-failed; tail -5 gpurun_out/agemm_bench.log; exit 1; }
grep shape gpurun_out/agemm_bench.log | python -c "import sys,json; [print(d['shape'],d['pass'],d['impl'],d['ms'],d['tflops'],d['vs_blaslt']) for d in map(json.loads,sys.stdin)]"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_asm.log 2>&1 || { echo e2e-asm-failed; tail -5 gpurun_out/bench_asm.log; exit 1; }
tail -1 gpurun_out/bench_asm.log | cut -c1-200
