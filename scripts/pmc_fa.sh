#!/bin/bash
# Per-kernel PMC passes over the flash-attention kernels at one shape (one counter group per
# rocprofv3 run). usage: scripts/pmc_fa.sh OUTDIR [SHAPE]
set -o pipefail
OUT=$1; SHAPE=${2:-"64,1024,16,128"}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 tools/bench_attn.py --no-sdpa --shapes "$SHAPE" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" fa_ > "$OUT/summary.txt" && cat "$OUT/summary.txt"
