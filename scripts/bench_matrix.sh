#!/bin/bash
# bench.py over the BASELINE.json configs that fit one GPU (run on the gpurun box)
set -o pipefail
TAG=${1:-m}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bm_${TAG}_base.json 2> gpurun_out/bm_${TAG}_base.err && \
timeout -k 10 300 python bench.py --model tiny --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bm_${TAG}_tiny.json 2> gpurun_out/bm_${TAG}_tiny.err && \
timeout -k 10 300 python bench.py --model small --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bm_${TAG}_small.json 2> gpurun_out/bm_${TAG}_small.err && \
timeout -k 10 300 python bench.py --model small-q5_1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bm_${TAG}_smallq5.json 2> gpurun_out/bm_${TAG}_smallq5.err && \
timeout -k 10 300 python bench.py --clips-per-gpu 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bm_${TAG}_base8.json 2> gpurun_out/bm_${TAG}_base8.err && \
timeout -k 10 500 python bench.py --model large-v3 --beam 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bm_${TAG}_lv3b5.json 2> gpurun_out/bm_${TAG}_lv3b5.err
timeout -k 10 400 python bench.py --model large-v3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bm_${TAG}_lv3.json 2> gpurun_out/bm_${TAG}_lv3.err
echo "EXIT $?"
