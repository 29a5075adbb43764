#!/bin/bash
# Skinny-GEMM config sweep (incl. the B-deep rings) at GPT-1.3B serving-batch decode shapes, bf16.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
S="8,6144,2048;8,8192,2048;8,2048,2048;8,2048,8192;16,6144,2048;16,8192,2048;16,2048,2048;16,2048,8192;32,6144,2048;32,8192,2048;32,2048,2048;32,2048,8192"
timeout -k 10 600 python tools/tune_small_gemm.py --dtype bf16 --shapes "$S" > gpurun_out/r6l_tune.jsonl 2> gpurun_out/r6l_tune.err || { tail -20 gpurun_out/r6l_tune.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r6l_tune.jsonl'):
    d=json.loads(l); print(d['M'],d['N'],d['K'],'best',d['best'],d['best_us'],'heur',d['heuristic'],d['heur_us'],'blaslt',d['hipblaslt_us'],'asm',d['asm_us'])
"
