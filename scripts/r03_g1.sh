#!/bin/bash
# round-3 first GPU session: seam/prefetch probe, decoder phase trace, the new
# host-logic tests, and the bench line with every single-GPU config
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 240 ./scripts/poll_probe > gpurun_out/poll_probe.txt 2>&1 && echo PROBE_OK && \
timeout -k 10 300 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/ptrace_r03a.log 2>&1 && echo TRACE_OK && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_timestamps.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "fault or beam_one or timestamp or transcribe or segment" > gpurun_out/t_r03a.log 2>&1 && echo TEST_OK && \
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err && echo BENCH_OK
