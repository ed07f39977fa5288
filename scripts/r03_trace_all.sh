#!/bin/bash
# final phase traces: base 1 row, base 8 rows, large-v3 5 rows
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/fin_tr1.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 8 > gpurun_out/fin_tr8.log 2>&1 || exit 1
timeout -k 10 400 python3 -u scripts/diag_persist.py trace large-v3 5 > gpurun_out/fin_lv5.log 2>&1 || exit 1
grep "wg 0: step" gpurun_out/fin_tr1.log gpurun_out/fin_tr8.log gpurun_out/fin_lv5.log
