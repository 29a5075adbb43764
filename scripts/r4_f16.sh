#!/bin/bash
set -o pipefail
cd /root/repo
timeout -k 10 200 python tools/probe_f16_gemm.py
