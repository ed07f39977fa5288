#!/bin/bash
# mel parity tests + the base bench (mel stage time), after a k_mel_frames change
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu -k "mel or checksum or encoder_micro or large_v3" > $O/mel_tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 $O/mel_tests.log; exit 1; }
tail -1 $O/mel_tests.log
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/mel_bench.log 2>&1 || { echo BENCH FAILED; exit 1; }
grep "^{" $O/mel_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/mel_trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/mel_trace.log 2>&1 || exit 1
grep -i mel_frames $GRAFT_REPO_ROOT/$O/mel_trace/run_kernel_stats.csv | cut -d, -f1-4
echo DONE
