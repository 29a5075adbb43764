#!/bin/bash
# Full GPU tier + smoke at HEAD.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_tier.log 2>&1 || { tail -40 gpurun_out/r6_tier.log; exit 1; }
tail -3 gpurun_out/r6_tier.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
