#!/bin/bash
# Decode mega kernel: FFN next-slice DMA at the GEMV midpoint vs after the GEMV.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 0 1; do
  echo "== late_dma $L"
  PIAMD_MEGA_LATE_DMA=$L timeout -k 10 200 python tools/mega_trace.py > gpurun_out/r4m_late_$L.log 2>&1 || { tail -20 gpurun_out/r4m_late_$L.log; exit 1; }
  grep "^{" gpurun_out/r4m_late_$L.log
done
