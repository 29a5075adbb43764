#!/bin/bash
# PMC A/B of the assembly NT GEMM vs hipBLASLt on the GPT-1.3B training shapes (one counter group per run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5_pmc_ab
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "list rc=$?"
for S in "98304 2048 2048" "98304 2048 8192" "98304 8192 2048"; do
  set -- $S
  timeout -k 10 120 python3 tools/gemm_ab_probe.py --M $1 --N $2 --K $3 --layout nt --iters 20 --rounds 5 >> $OUT/wall.jsonl 2>&1 || { echo "wall failed"; tail -5 $OUT/wall.jsonl; exit 1; }
done
cat $OUT/wall.jsonl
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 tools/gemm_ab_probe.py --M 98304 --N 2048 --K 2048 --iters 10 --rounds 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
