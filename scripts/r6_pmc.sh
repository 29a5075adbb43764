#!/bin/bash
# PMC passes over the assembly dK/dV kernel at the bench shape (one counter group per run).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_pmc
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH"
P4="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P5="SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INSTS_WAVE32_LDS SQ_IFETCH SQ_INSTS_VALU_CVT SQ_WAVE_CYCLES"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  PIAMD_FA_ASM=1 timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 tools/bench_attn.py --no-sdpa --shapes "96,1024,16,128" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" dkdv > "$OUT/summary.txt" && cat "$OUT/summary.txt"
