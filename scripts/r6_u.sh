#!/bin/bash
# FA ring-lookahead variants (dQ QLA 4 / 8, forward F_LA 3 / 6 vs defaults 6 / 4): correctness + per-kernel times at B96 S1024.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6u
for V in default qla4 qla8 fla6 fla3; do
  if [ $V = default ]; then H=$R/paddle_infer_amd/_lib/piamd_fa.hsaco; else H=$R/paddle_infer_amd/_lib/fa_$V.hsaco; fi
  PIAMD_FA_HSACO=$H timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fa_asm_gpu.py > gpurun_out/r6u/t_$V.log 2>&1 || { echo "$V tests FAILED"; tail -15 gpurun_out/r6u/t_$V.log; exit 1; }
  echo "$V: $(tail -1 gpurun_out/r6u/t_$V.log)"
  (cd /tmp && PIAMD_FA_HSACO=$H timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/r6u/p_$V -o run -- python $R/tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > $R/gpurun_out/r6u/p_$V.log 2>&1) || { tail -20 gpurun_out/r6u/p_$V.log; exit 1; }
  python tools/rocpd_stats.py $(ls gpurun_out/r6u/p_$V/*/*.db gpurun_out/r6u/p_$V/*.db 2>/dev/null | head -1) --top 6 > gpurun_out/r6u/s_$V.txt 2>&1 || true
  grep -E "piamd_fa" gpurun_out/r6u/s_$V.txt | cut -c1-130
  rm -rf gpurun_out/r6u/p_$V
done
