#!/bin/bash
# Pricing the operand path: ablated assembly-GEMM variants on the out-projection shape.
#   vload: LDS-DMA -> plain VMEM loads into scratch VGPRs; dsw: -> ds_write_b128 of a fixed register;
#   mfma32: 32x32x16 MFMAs (half the count) at the same slots. Timing only (results are garbage).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_g
mkdir -p $OUT
for V in base nodma vload vload+dsw dsw mfma32 mfma32+nodma; do
  if [ $V = base ]; then H=paddle_infer_amd/_lib/piamd_agemm.hsaco; else H=paddle_infer_amd/_lib/piamd_agemm_abl_$V.hsaco; fi
  PIAMD_AGEMM_HSACO=$H timeout -k 10 120 python3 tools/gemm_ab_probe.py --M 98304 --N 2048 --K 2048 --impls asm --iters 20 --rounds 5 > $OUT/wall_$V.jsonl 2>&1 || { echo "wall $V failed"; tail -3 $OUT/wall_$V.jsonl; exit 1; }
  echo "$V $(grep '^{' $OUT/wall_$V.jsonl)"
  PIAMD_AGEMM_HSACO=$H timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d "$OUT/p_$V" -o run --output-format csv -- python3 tools/gemm_ab_probe.py --M 98304 --N 2048 --K 2048 --impls asm --iters 10 --rounds 1 > "$OUT/p_$V.log" 2>&1 || { echo "pmc $V failed"; exit 1; }
  python3 tools/pmc_summary.py $OUT/p_$V agemm | grep -E "GRBM_GUI|WAVE_CYCLES|WAIT" 
done
