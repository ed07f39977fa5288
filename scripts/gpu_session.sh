#!/bin/bash
# Session check on the gpurun box: GPU parity tests, bench (base), decoder
# timeline (WMI_TRACE), rocprofv3 kernel stats.  Every GPU step is time-limited
# and chained with &&: nothing more runs on the GPU after a failure.
# Usage (repo root on the box): bash scripts/gpu_session.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-s}
shift
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/tests_$TAG.log 2>&1 && echo "PYTEST ok" && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
echo "BENCH ok" && \
WMI_TRACE=1 timeout -k 10 120 python scripts/probe.py base 16 > gpurun_out/trace_$TAG.log 2>&1 && echo "TRACE ok" && \
cd /tmp && export TMPDIR=/tmp && WMI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
echo "EXIT $?"
