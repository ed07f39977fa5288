#!/bin/bash
# phase traces of the multi-row instances: base x 8 rows, large-v3 x 5 rows
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 8 > gpurun_out/mr_tr8.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/mr_tr8.log | head -24
timeout -k 10 400 python3 -u scripts/diag_persist.py trace large-v3 5 > gpurun_out/mr_lv5.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/mr_lv5.log | head -24
