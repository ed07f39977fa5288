#!/bin/bash
# round-3 GPU session: seam/prefetch probe, decoder phase trace, the GPU test
# suite, and the bench line with every single-GPU config
set -o pipefail
TAG=${1:-r03a}
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 240 ./scripts/poll_probe > gpurun_out/poll_probe.txt 2>&1 && echo PROBE_OK && \
timeout -k 10 300 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/ptrace_$TAG.log 2>&1 && echo TRACE_OK && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_$TAG.log 2>&1 && echo TEST_OK && \
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && echo BENCH_OK
