#!/bin/bash
# A/B of the encoder attention kernels (WMI_ENC_ATTN=3: 32-query blocks;
# 4: LDS-shared K/V, three sweeps; WMI_ENC_ATTN_NW waves per workgroup) at 1
# and 8 base clips, after the encoder parity tests on the default kernel.
# Run on the gpurun box from the repo root.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "encoder or batch or full_size or large_v3 or f32" > $O/attn_tests.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
for clips in 1 8; do
  for cfg in "3 0" "4 2" "4 4"; do
    set -- $cfg
    WMI_ENC_ATTN=$1 WMI_ENC_ATTN_NW=$2 timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --clips-per-gpu $clips \
      > $O/attn_ab_c${clips}_v$1_nw$2.log 2>&1 || { echo "BENCH FAILED $clips $cfg"; exit 1; }
    python3 - $O/attn_ab_c${clips}_v$1_nw$2.log "clips $clips enc_attn v$1 nw $2" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
k = d["kernels"]["enc_attn"]
print(f"{sys.argv[2]}: {k['avg_us']:.1f} us ({k['TFLOP/s']:.0f} TF/s); encoder_ms {d['encoder_ms']}; value {d['value']}")
PY
  done
done
echo DONE
