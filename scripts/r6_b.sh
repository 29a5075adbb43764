#!/bin/bash
# Round 6: new GPU tests (colsum epilogue, SyncBN kernels, RCCL world-1, HIP graph API) + fused-db1 A/B bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_agemm_gpu.py tests/test_sync_batchnorm_gpu.py tests/test_rccl_world1_gpu.py tests/test_cuda_graph_api_gpu.py tests/test_conv3d_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  PIAMD_FUSED_DB1=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_db1_$v.log 2>&1 || { tail -20 $OUT/bench_db1_$v.log; exit 1; }
  echo "db1=$v $(tail -1 $OUT/bench_db1_$v.log | cut -c1-200)"
done
