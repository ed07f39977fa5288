#!/bin/bash
# logits GEMV grid sweep (run on the gpurun box after the parity tests)
set -o pipefail
mkdir -p gpurun_out
for cap in 256 512 768 1024; do
  WMI_LOGITS_CAP=$cap timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tl_base_$cap.json 2>/dev/null || exit 1
  WMI_LOGITS_CAP=$cap timeout -k 10 200 python bench.py --model small-q5_1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tl_q5_$cap.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --model small --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tl_small.json 2>/dev/null
