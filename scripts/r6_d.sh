#!/bin/bash
# Round 6: bench + census with the assembly FA backward, then the GEMM clock/power table.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/bench_prof.sh r6fa || exit 1
for s in 8192,8192,8192 24576,2048,8192; do
  timeout -k 10 120 python tools/gemm_power.py $s 4 >> gpurun_out/gemm_power.jsonl 2>gpurun_out/gemm_power.err || { tail -5 gpurun_out/gemm_power.err; exit 1; }
done
cat gpurun_out/gemm_power.jsonl
