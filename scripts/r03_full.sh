#!/bin/bash
# full -m gpu suite, base trace, default bench line (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/trace_$TAG.log 2>&1 || exit 1
grep -v "wg G/2" gpurun_out/trace_$TAG.log | head -24
timeout -k 10 300 python3 bench.py --configs none --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['stage_ms'], d['roofline']['frac'])"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/ -m gpu > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -n 3 gpurun_out/tests_$TAG.log; exit $rc
