#!/bin/bash
# multi-row poll width 32 (main) vs 16 (pu16): decoder tests, C4 shard and C5
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -k "batch or persistent_matches or persistent_beam or beam_shared or persistent_q5 or beam_search" > gpurun_out/pu_t.log 2>&1; rc=$?; tail -n 2 gpurun_out/pu_t.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in main pu16; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 300 python3 bench.py --clips-per-gpu 8 --configs none --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abpu.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abpu.json')); print('$v base x8', d['value'], d['stage_ms']['decode_ms'])"
  timeout -k 10 300 python3 bench.py --model large-v3 --beam 5 --configs none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/abpu.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abpu.json')); print('$v lv3 beam5', d['value'], d['stage_ms']['decode_ms'])"
done; done
