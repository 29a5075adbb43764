#!/bin/bash
# asm GEMM tile-group (GROUP_M) and persistent-mode sweep on the training shapes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for CFG in "8 0" "4 0" "16 0" "32 0" "8 1"; do
  set -- $CFG
  if [ "$2" = "1" ]; then export PIAMD_AGEMM_NO_PERSIST=1; else unset PIAMD_AGEMM_NO_PERSIST; fi
  PIAMD_AGEMM_GM=$1 timeout -k 10 200 python tools/agemm_check.py --stage bench > gpurun_out/agemm_gm_$1_$2.log 2>&1 || { tail -5 gpurun_out/agemm_gm_$1_$2.log; exit 1; }
  echo "== GM $1 nopersist $2"
  grep '"impl": "asm' gpurun_out/agemm_gm_$1_$2.log | python3 -c "
import sys, json
rows=[json.loads(l) for l in sys.stdin]
print(' '.join(f\"{r['shape']}/{r['pass']}={r['ms']:.3f}\" for r in rows), ' total=%.2f' % sum(r['ms'] for r in rows))"
done
