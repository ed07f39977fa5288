#!/bin/bash
# traces (1 and 8 rows) and bench at 1 and 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/tb_tr1_$TAG.log 2>&1 || exit 1
grep "wg 0" gpurun_out/tb_tr1_$TAG.log | head -3; grep "logits" gpurun_out/tb_tr1_$TAG.log | head -1
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 8 > gpurun_out/tb_tr8_$TAG.log 2>&1 || exit 1
grep "wg 0" gpurun_out/tb_tr8_$TAG.log | head -3; grep "logits" gpurun_out/tb_tr8_$TAG.log | head -1
for cpg in 1 8; do
  timeout -k 10 200 python3 bench.py --configs none --no-cpu-baseline --steps 5 --warmup 2 --clips-per-gpu $cpg > gpurun_out/tb_b${cpg}_$TAG.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/tb_b${cpg}_$TAG.json')); print('cpg $cpg', d['value'], d['stage_ms']['decode_ms'], d['roofline']['frac'])"
done
