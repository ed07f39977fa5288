#!/bin/bash
# One GPU round on the gpurun box: parity tests, bench, rocprofv3 kernel trace.
# Usage (from the repo root on the box): bash scripts/gpu_round.sh TAG
# Writes gpurun_out/{tests,bench,prof}_TAG*.  Each GPU step has its own time
# limit and the steps are chained: nothing more runs on the GPU after a failure.
set -o pipefail
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/tests_$TAG.log 2>&1
echo "PYTEST $?"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && WMI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
echo "EXIT $?"
