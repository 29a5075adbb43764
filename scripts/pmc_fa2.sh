#!/bin/bash
# PMC passes over the FA kernels for bwd v1 and v2 at the bench shape (one counter group per run).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in 1 2; do
  PIAMD_FA_BWD_V=$V bash scripts/pmc_fa.sh gpurun_out/pmc_fa_v$V "96,1024,16,128" > gpurun_out/pmc_fa_v$V.txt 2>&1 || { tail -5 gpurun_out/pmc_fa_v$V.txt; exit 1; }
done
