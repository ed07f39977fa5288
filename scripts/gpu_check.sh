#!/bin/bash
# Standard GPU round-trip after a decoder change (run on the gpurun box from
# the repo root): the base phase trace, the bench line, the -m gpu suite.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag_persist.py trace ${TRACE_MODEL:-base} ${TRACE_ROWS:-1} > $O/trace_chk.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_chk.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/ -m gpu > $O/gpu_chk.log 2>&1
echo "EXIT $?"
