#!/bin/bash
# round-3 session-2 baseline: -m gpu suite, then the default bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/ -m gpu > $O/s2_tests.log 2>&1; echo "TESTS $?"
tail -3 $O/s2_tests.log
timeout -k 10 600 python3 bench.py > $O/s2_bench.json 2> $O/s2_bench.err; echo "BENCH $?"
tail -c 600 $O/s2_bench.json
