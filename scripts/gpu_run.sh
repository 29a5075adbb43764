#!/bin/bash
# Runs a list of GPU steps, each under its own timeout; stops at the first crash / timeout
# (exit >= 124 or signal), continues past ordinary failures (e.g. pytest exit 1).
# usage: scripts/gpu_run.sh "<timeout> <name> <cmd...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  t=$(echo "$spec" | awk '{print $1}')
  name=$(echo "$spec" | awk '{print $2}')
  cmd=$(echo "$spec" | cut -d' ' -f3-)
  echo "=== [$name] ($t s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc ($(( $(date +%s) - start )) s)"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP: $name crashed/timed out (rc=$rc)"; exit $rc; fi
done
exit 0
