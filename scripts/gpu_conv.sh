#!/bin/bash
# Conv coverage: direct grouped/depthwise kernels, fp16 MFMA conv, 1x1 GEMM route, NCHW, MobileNetV2.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_conv_any_gpu.py tests/test_conv_gpu.py tests/test_conv_bwd_gpu.py > gpurun_out/conv_any.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/conv_any.log | tail -60
exit $rc
