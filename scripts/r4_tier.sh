#!/bin/bash
# Full GPU tier (what the driver runs at round end) + smoke + a short bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t_tier.log 2>&1 || { tail -60 gpurun_out/r4t_tier.log; exit 1; }
tail -3 gpurun_out/r4t_tier.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
