#!/bin/bash
# base phase trace (sub-stamps in B and F) and one bench line
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-t1}
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/trace_$TAG.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/trace_$TAG.log | head -40
