#!/bin/bash
# phase traces: base with 8 rows (C4's shard), large-v3 with 1 row
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 8 > gpurun_out/trace8_$TAG.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/trace8_$TAG.log | head -24
timeout -k 10 400 python3 -u scripts/diag_persist.py trace large-v3 1 > gpurun_out/tracelv3_$TAG.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/tracelv3_$TAG.log | head -24
