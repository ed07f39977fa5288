#!/bin/bash
# poll backoff and computed-exp encoder attention, against the in-tree build
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
bash scripts/ab_lib.sh s2 main sleep1 cexp main sleep1 cexp || exit 1
WMI_LIB=$PWD/whisper.rs_amd/ab/cexp/libwhisper_mi355x.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "enc_attn or encoder or exp" > gpurun_out/cexp_tests.log 2>&1; echo "CEXP TESTS $?"; tail -n 2 gpurun_out/cexp_tests.log
for cpg in 8; do
 for v in main cexp; do
  if [ $v = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --configs none --no-cpu-baseline --clips-per-gpu $cpg > gpurun_out/s2_b8_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/s2_b8_$v.json')); print('$v x8', d['value'], d['encoder_ms'], d['kernels']['enc_attn'])"
 done
done
