#!/bin/bash
# q5_1 weights dequantised inside the polls: parity tests, then C3 (small
# q5_1, 1 clip) with and without the q5_1 GEMVs, and 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_quant.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "q5 or quantised" > gpurun_out/q5_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/q5_tests.log; [ $rc -eq 0 ] || exit 1
MODEL=small-q5_1 bash scripts/ab.sh "WMI_PERSIST_Q5=1" "WMI_PERSIST_Q5=0" "WMI_PERSIST_Q5=1" "WMI_PERSIST_Q5=0" || exit 1
MODEL=small-q5_1 CPG=8 bash scripts/ab.sh "WMI_PERSIST_Q5=1" "WMI_PERSIST_Q5=0" || exit 1
bash scripts/ab.sh "WMI_X=0" || exit 1
