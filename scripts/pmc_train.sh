#!/bin/bash
# One PMC pass (8 SQ counters, known-valid names) over a short GPT-3 1.3B-shaped training run
# (4 layers, micro-batch 64: the real per-layer GEMM / attention / LN shapes): MFMA-busy and
# wait fractions per kernel. Counters only (no trace domains), bounded by timeout -s KILL.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_train
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $P1 -d "$OUT/p1" -o run --output-format csv -- python3 bench.py --num-layers 4 --micro-batch 64 --steps 1 --warmup 1 > "$OUT/p1.log" 2>&1 || { echo "pmc pass failed rc=$?"; tail -5 "$OUT/p1.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
find "$OUT" -name "*.csv" -delete
head -80 "$OUT/summary.txt"
