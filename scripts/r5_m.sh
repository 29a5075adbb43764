#!/bin/bash
# Native device runtime (streams / events / properties / tracer) + GPU tests touching streams.
set -o pipefail
OUT=gpurun_out/r5_m
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_device_runtime_gpu.py tests/test_allocator_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
