#!/bin/bash
# A/B timing of decoder variants on the gpurun box: bench.py (base unless
# MODEL is set), 3 steps each; each line "<env> value decode_ms logits_us".
# MODEL / BEAM / CPG select the config (default base, greedy, 1 clip).
# Usage: bash scripts/ab.sh "ENV=1 ENV2=0" "ENV=0" ...
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
MODEL=${MODEL:-base}
BEAM=${BEAM:-0}
CPG=${CPG:-1}
for v in "$@"; do
  timeout -k 10 200 env $v python bench.py --model $MODEL --beam $BEAM --clips-per-gpu $CPG --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['stage_ms']['decode_ms'], d['encoder_ms'], d['roofline']['avg_us'])" || exit 1
done
echo "AB EXIT 0"
