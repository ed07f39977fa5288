#!/bin/bash
# Full GPU suite, then the base bench (1 clip; 8 clips with enc3 / enc4) and a
# kernel-trace of the 1-clip bench.  Run on the gpurun box from the repo root.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/c2_tests.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_bench1.log 2>&1 || { echo "BENCH1 FAILED"; exit 1; }
for v in 3 4; do
  WMI_ENC_ATTN=$v timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --clips-per-gpu 8 > $O/c2_bench8_v$v.log 2>&1 || { echo "BENCH8 FAILED"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c2_trace.log 2>&1 || { echo "TRACE FAILED"; exit 1; }
echo "EXIT 0"
