#!/bin/bash
# MFMA GEMVs at every n for several rows (main) vs n <= 512 (m512): tests, large-v3 5 beams, small x 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -k "large_v3 or beam_shared or persistent_beam or q5 or beam_search" > gpurun_out/mgvl_t.log 2>&1; rc=$?; tail -n 2 gpurun_out/mgvl_t.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in main m512; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 300 python3 bench.py --model large-v3 --beam 5 --configs none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/abm.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abm.json')); print('$v lv3 beam5', d['value'], d['stage_ms']['decode_ms'])"
  timeout -k 10 300 python3 bench.py --model small --clips-per-gpu 8 --configs none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/abm.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abm.json')); print('$v small x8', d['value'], d['stage_ms']['decode_ms'])"
done; done
