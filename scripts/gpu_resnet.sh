#!/bin/bash
# ResNet-50: BN/conv tests, eager + hipGraph throughput, BN grid A/B, kernel profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_attention_gpu.py tests/test_conv_any_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_gpu.py tests/test_norm_gpu.py > gpurun_out/rn_tests.log 2>&1 || { tail -40 gpurun_out/rn_tests.log; exit 1; }
tail -1 gpurun_out/rn_tests.log
timeout -k 10 300 python tools/bench_resnet.py --steps 10 > gpurun_out/resnet_e.log 2>&1 || { tail -20 gpurun_out/resnet_e.log; exit 1; }
grep "^{" gpurun_out/resnet_e.log
timeout -k 10 300 python tools/bench_resnet.py --steps 10 --graph > gpurun_out/resnet_g.log 2>&1 || { tail -30 gpurun_out/resnet_g.log; exit 1; }
grep "^{" gpurun_out/resnet_g.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet2 -o run -- python tools/bench_resnet.py --steps 3 > gpurun_out/prof_resnet2.log 2>&1 || { tail -20 gpurun_out/prof_resnet2.log; exit 1; }
echo done
