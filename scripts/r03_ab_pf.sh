#!/bin/bash
# L2 warm-up (main) vs none (nopf): large-v3 greedy and 5-beam, alternating
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "large_v3 or beam_shared" > gpurun_out/pf_t.log 2>&1; rc=$?; tail -n 2 gpurun_out/pf_t.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in main nopf; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 300 python3 bench.py --model large-v3 --configs none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/abpf.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abpf.json')); print('$v greedy', d['value'], d['stage_ms']['decode_ms'])"
  timeout -k 10 300 python3 bench.py --model large-v3 --beam 5 --configs none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/abpf.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abpf.json')); print('$v beam5', d['value'], d['stage_ms']['decode_ms'])"
done; done
