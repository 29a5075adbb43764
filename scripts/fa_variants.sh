#!/bin/bash
# FA timing across kernel-library variants in _lib/ab (libpiamd_kernels_<name>.so) + the in-tree
# build ("new"). usage: scripts/fa_variants.sh "SHAPES" name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
SHAPES=$1; shift
mkdir -p gpurun_out
for v in "$@" new; do
  if [ $v = new ]; then unset PIAMD_KERNEL_LIB; else export PIAMD_KERNEL_LIB=$PWD/paddle_infer_amd/_lib/ab/libpiamd_kernels_$v.so; fi
  echo "== $v"
  timeout -k 10 180 python tools/bench_attn.py --no-sdpa --shapes "$SHAPES" 2>/dev/null | grep "^{" | cut -c1-220 || exit 1
done
