#!/bin/bash
# HEAD check: full GPU tier, smoke, 1-GPU bench, decode at prompt 128 / 1024, ResNet ATen trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6f_tier.log 2>&1 || { tail -40 gpurun_out/r6f_tier.log; exit 1; }
tail -2 gpurun_out/r6f_tier.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f_smoke.log 2>&1 || { tail -20 gpurun_out/r6f_smoke.log; exit 1; }
tail -1 gpurun_out/r6f_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6f_bench.log 2>&1 || { tail -30 gpurun_out/r6f_bench.log; exit 1; }
grep '^{' gpurun_out/r6f_bench.log
for p in 1024 128; do
  timeout -k 10 200 python tools/bench_generate.py --batch 1 --prompt $p --gen 128 --modes graph > gpurun_out/r6f_dec_$p.log 2>&1 || { tail -20 gpurun_out/r6f_dec_$p.log; exit 1; }
  echo "prompt=$p"; grep '^{' gpurun_out/r6f_dec_$p.log
done
true
