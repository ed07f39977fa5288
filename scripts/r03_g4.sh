#!/bin/bash
# encoder parity with the |device - exact| bar, the LDS-K/V bitwise test, and
# phase traces of the several-row (BT = 8) persistent decoder at large-v3
set -o pipefail
TAG=${1:-r03h}
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "encoder or lds_kv or full_size or small_q5 or large_v3" > gpurun_out/t1_$TAG.log 2>&1 && echo TEST1_OK && \
timeout -k 10 300 python3 -u scripts/diag_persist.py trace large-v3 5 > gpurun_out/ptrace_lv3x5_$TAG.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/diag_persist.py trace large-v3 1 > gpurun_out/ptrace_lv3x1_$TAG.log 2>&1 && echo TRACE_OK
