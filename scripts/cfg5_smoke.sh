#!/bin/bash
# BASELINE config-5 path on one GPU: GPT-3 13B architecture (4 of its 40 layers), ZeRO-3 through
# fleet (sharding stage 3, world 1), with and without host offload of the optimizer states.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --model gpt3-13b --num-layers 4 --micro-batch 8 --sharding 3 --steps 3 --warmup 1 > gpurun_out/cfg5_s3.log 2>&1 || { tail -20 gpurun_out/cfg5_s3.log; exit 1; }
tail -1 gpurun_out/cfg5_s3.log | cut -c1-400
timeout -k 10 400 python bench.py --model gpt3-13b --num-layers 4 --micro-batch 8 --sharding 3 --offload 1 --steps 3 --warmup 1 > gpurun_out/cfg5_s3_off.log 2>&1 || { tail -20 gpurun_out/cfg5_s3_off.log; exit 1; }
tail -1 gpurun_out/cfg5_s3_off.log | cut -c1-400
