#!/bin/bash
# Full GPU tier + MobileNetV2 / ResNet-50 throughput and MobileNetV2 kernel trace (autocast linears on own GEMMs).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t2_tier.log 2>&1 || { tail -60 gpurun_out/r4t2_tier.log; exit 1; }
tail -2 gpurun_out/r4t2_tier.log
for M in resnet50 mobilenet_v2; do
  timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4t2_cn_$M.log 2>&1 || { tail -20 gpurun_out/r4t2_cn_$M.log; exit 1; }
  grep "^{" gpurun_out/r4t2_cn_$M.log | cut -c1-200
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4t2_prof_mbv2 -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --model mobilenet_v2 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4t2_prof_mbv2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4t2_prof_mbv2 > gpurun_out/r4t2_prof_mbv2.txt 2>&1
head -20 gpurun_out/r4t2_prof_mbv2.txt
echo "Cijk rows: $(grep -c Cijk gpurun_out/r4t2_prof_mbv2.txt || true)"
