#!/bin/bash
# End-of-round check (run on the gpurun box from the repo root): the -m gpu
# suite, then the round-2 measurement set (bench line with CPU baseline,
# rocprofv3 kernel table of the bench command, FETCH/WRITE passes over the
# persistent decoder) and the 8-clip C4 shard bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/r02b_tests.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
tail -1 $O/r02b_tests.log
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --clips-per-gpu 8 > $O/r02b_bench8.log 2>&1 || { echo "BENCH8 FAILED"; exit 1; }
bash $R/scripts/r02_measure.sh || exit 1
echo "ALL DONE"
