#!/bin/bash
# MFMA logits: decoder parity tests, traces (1 and 8 rows), bench 1 and 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "teacher_forced or logits_full or greedy or batch or persistent or beam_search or beam_one or staged or full_size or timeout or q5" \
  > gpurun_out/lmf_t_$TAG.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/lmf_t_$TAG.log | tail -n 2; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/lmf_tr1_$TAG.log 2>&1 || exit 1
grep "step\|logits" gpurun_out/lmf_tr1_$TAG.log | head -4
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 8 > gpurun_out/lmf_tr8_$TAG.log 2>&1 || exit 1
grep "step\|logits" gpurun_out/lmf_tr8_$TAG.log | head -4
for cpg in 1 8; do
  timeout -k 10 200 python3 bench.py --configs none --no-cpu-baseline --steps 5 --warmup 2 --clips-per-gpu $cpg > gpurun_out/lmf_b${cpg}_$TAG.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/lmf_b${cpg}_$TAG.json')); print('cpg $cpg', d['value'], d['stage_ms']['decode_ms'], d['roofline']['frac'])"
done
