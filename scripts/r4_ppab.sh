#!/bin/bash
# A/B of the ping-pong GEMM schedule variants against the 4-wave kernel (NT fwd/dgrad, GPT shapes)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
run() {  # $1 = label, rest = env
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u tools/agemm_check.py --stage bench --rounds 3 --shapes out,ffn1,ffn2 > gpurun_out/r4_ab_$lab.jsonl 2>&1 || { tail -20 gpurun_out/r4_ab_$lab.jsonl; return 1; }
  echo "== $lab"; grep '"asm"' gpurun_out/r4_ab_$lab.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['pass'], d['tflops'], d['vs_blaslt'])"
}
run old PIAMD_AGEMM_PP=0 && run pp PIAMD_AGEMM_PP=1 && run v1 PIAMD_AGEMM_PP=1 PIAMD_AGEMM_PPV=1 && run v2 PIAMD_AGEMM_PP=1 PIAMD_AGEMM_PPV=2 && run v3 PIAMD_AGEMM_PP=1 PIAMD_AGEMM_PPV=3
