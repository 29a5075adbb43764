#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "conv or infer or predictor or resnet or mobilenet or static" > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/conv_nets.sh
