#!/bin/bash
# full -m gpu suite, then encoder attention NW A/B (1 clip and 8 clips)
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 1100 python3 -u -m pytest -x -v -s -k "large_v3 or not full_size" --timeout 700 --timeout-method thread tests/ -m gpu > gpurun_out/tests_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|compared over" gpurun_out/tests_$TAG.log | tail -n 3; [ $rc -eq 0 ] || exit 1
for nw in 0 1 2; do for cpg in 1 8; do
  WMI_ENC_ATTN_NW=$nw timeout -k 10 200 python3 bench.py --configs none --no-cpu-baseline --steps 3 --warmup 1 --clips-per-gpu $cpg > gpurun_out/nw_${nw}_$cpg.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/nw_${nw}_$cpg.json')); print('nw $nw cpg $cpg', d['value'], d['encoder_ms'], d['kernels']['enc_attn'])"
done; done
