#!/bin/bash
# decoder tests, then MFMA logits (main) vs VALU logits (xqfm), alternating, 1 and 8 clips
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_timestamps.py tests/test_dist_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -k "teacher_forced or logits_full or greedy or batch or persistent or beam or staged or timeout or q5 or lds or timestamp or rccl or transcribe" \
  > gpurun_out/xq_t.log 2>&1; rc=$?; tail -n 2 gpurun_out/xq_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/xq_tr1.log 2>&1 || exit 1
grep "wg 0" gpurun_out/xq_tr1.log | head -3; grep "logits" gpurun_out/xq_tr1.log | head -1
for rep in 1 2; do for v in main xqfm; do for cpg in 8; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 200 python3 bench.py --configs none --no-cpu-baseline --steps 5 --warmup 2 --clips-per-gpu $cpg > gpurun_out/abxq.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abxq.json')); print('$v cpg $cpg', d['value'], d['stage_ms']['decode_ms'])"
done; done; done
for v in main xqfm; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 300 python3 bench.py --model tiny --beam 5 --configs none --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abxq.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abxq.json')); print('$v tiny beam5', d['value'], d['stage_ms']['decode_ms'])"
done
