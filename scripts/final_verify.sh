#!/bin/bash
# Last check of the round's tree: -m gpu suite, smoke, then the measurement set.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/fv_tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 $O/fv_tests.log; exit 1; }
tail -1 $O/fv_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/fv_smoke.log 2>&1 || { echo "SMOKE FAILED"; exit 1; }
tail -1 $O/fv_smoke.log
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --clips-per-gpu 8 > $O/fv_bench8.log 2>&1 || { echo "BENCH8 FAILED"; exit 1; }
bash $R/scripts/r02_measure.sh
