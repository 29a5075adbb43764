#!/bin/bash
# FA forward: 4 vs 8 waves per workgroup — correctness (attention GPU tests at 8 waves) + bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PIAMD_FA_FWD_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/fa8_test.log 2>&1 || { tail -30 gpurun_out/fa8_test.log; exit 1; }
tail -1 gpurun_out/fa8_test.log
for nw in 4 8; do
  PIAMD_FA_FWD_WAVES=$nw timeout -k 10 300 python tools/bench_attn.py --shapes "96,1024,16,128;8,2048,16,128;4,4096,16,128" --no-sdpa > gpurun_out/fa_nw$nw.log 2>&1 || { tail -20 gpurun_out/fa_nw$nw.log; exit 1; }
  echo "== waves $nw"; grep "^{" gpurun_out/fa_nw$nw.log | cut -c1-250
done
