#!/bin/bash
# MFMA logits (main) vs VALU logits (novlm), alternating, 1 and 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
for rep in 1 2 3; do for v in main novlm; do for cpg in 1 8; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 200 python3 bench.py --configs none --no-cpu-baseline --steps 5 --warmup 2 --clips-per-gpu $cpg > gpurun_out/ablmf.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ablmf.json')); print('$v cpg $cpg', d['value'], d['stage_ms']['decode_ms'])"
done; done; done
