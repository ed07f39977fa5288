#!/bin/bash
# Round-2 measurement set for the bench command (run on the gpurun box from
# the repo root): the bench line with its CPU baseline, the rocprofv3 kernel
# table of the same command, and FETCH_SIZE / WRITE_SIZE passes over the
# persistent decoder (wmi_bench_kernel 14) at the bench's 128 tokens.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 400 python3 -u $R/bench.py --steps 10 --warmup 3 > $O/r02_bench.json 2> $O/r02_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r02_prof_bench -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r02_prof_bench.log 2>&1 && \
bash $R/scripts/pmc_pass.sh persist base 14 3 128
echo "EXIT $?"
