#!/bin/bash
# Round-3 measurement set: the rocprofv3 kernel table of the bench command,
# then FETCH_SIZE / WRITE_SIZE passes over the persistent decoder
# (wmi_bench_kernel 14) at the bench's 128 tokens, then the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 200 python3 $R/bench.py --configs none --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03_prof_bench -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --configs none --no-cpu-baseline > $O/r03_prof_bench.log 2>&1 && \
bash $R/scripts/pmc_pass.sh persist3 base 14 3 128 && \
python3 $R/scripts/pmc_summary.py $O/pmc_persist3_fetch/run_counter_collection.csv $O/pmc_persist3_write/run_counter_collection.csv \
  "k_dec_persist<512, 1," $O/r03_pmc_persist_base.json "round-3 final build, base, 1 clip, 131 steps per launch" && \
cd $R && timeout -k 10 800 python3 bench.py > $O/r03_bench.json 2> $O/r03_bench.err
echo "EXIT $?"
