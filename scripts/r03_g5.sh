#!/bin/bash
# beam-shared cross-attention tasks (configs[4]): tests, then C5 bench with
# and without the sharing
set -o pipefail
TAG=${1:-r03i}
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 600 --timeout-method thread \
  -k "beam or large_v3" > gpurun_out/t1_$TAG.log 2>&1 && echo TEST1_OK && \
timeout -k 10 300 python3 bench.py --model large-v3 --beam 5 --steps 2 --warmup 1 --configs none --no-cpu-baseline \
  > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err && echo C5_OK && \
WMI_XSHARE=0 timeout -k 10 300 python3 bench.py --model large-v3 --beam 5 --steps 2 --warmup 1 --configs none --no-cpu-baseline \
  > gpurun_out/c5_noshare_$TAG.json 2> gpurun_out/c5_noshare_$TAG.err && echo C5NS_OK
