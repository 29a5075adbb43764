#!/bin/bash
set -o pipefail
bash scripts/r5_e.sh || exit 1
bash scripts/r5_d.sh
