#!/bin/bash
set -o pipefail
cd /root/repo
PIAMD_AGEMM_PP=1 timeout -k 10 120 python -u tools/pp_debug.py 2>&1 | grep -v amdgpu.ids
