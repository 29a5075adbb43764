#!/bin/bash
# ATen ops left in a ResNet-50 training step (operand shapes for the autograd engine's adds).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/trace_aten_step.py --model resnet50 --batch 128 > gpurun_out/r6r_trace.txt 2>&1 || { tail -20 gpurun_out/r6r_trace.txt; exit 1; }
head -50 gpurun_out/r6r_trace.txt | cut -c1-220
