#!/bin/bash
# round-3 verification: -m gpu suite, smoke, the default bench line (all configs + CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
TAG=${1:-x}
timeout -k 10 1100 python3 -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/ -m gpu > gpurun_out/fin_tests_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|compared over" gpurun_out/fin_tests_$TAG.log | tail -n 3; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke_$TAG.log 2>&1 || exit 1
tail -n 1 gpurun_out/fin_smoke_$TAG.log
timeout -k 10 800 python3 bench.py > gpurun_out/fin_bench_$TAG.json 2> gpurun_out/fin_bench_$TAG.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/fin_bench_$TAG.json')); print('bench', d['value'], d['stage_ms'], d['roofline']['frac'])
[print(k, v.get('audio_s_per_s'), v.get('decode_ms'), v.get('encoder_ms')) for k, v in d.get('configs', {}).items()]"
