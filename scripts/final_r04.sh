#!/bin/bash
# Round-4 closing run on the gpurun box: GPU suite + smoke + the driver's bench
# line + rocprof kernel table + PMC passes of the roofline kernel, each under
# its own limit (scripts/session.sh), then the PMC summary for bench.py.
set -o pipefail
T=${1:-fin}
bash scripts/session.sh $T tests smoke bench prof pmc=base:1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/${T}_pmc_base_1_fetch/run_counter_collection.csv \
  gpurun_out/${T}_pmc_base_1_write/run_counter_collection.csv "k_dec_persist<512, 1," \
  gpurun_out/${T}_pmc_persist_base.json "round-4 final build, base, 1 clip, 131 steps per launch" || exit 1
cat gpurun_out/${T}_pmc_persist_base.json
