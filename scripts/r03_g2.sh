#!/bin/bash
set -o pipefail
TAG=${1:-r03b}
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_$TAG.log 2>&1 && echo TEST_OK && \
bash scripts/ab_lib.sh $TAG main env:WMI_KVL=0
