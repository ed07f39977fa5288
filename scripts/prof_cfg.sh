#!/bin/bash
# rocprofv3 kernel-trace summaries of bench.py at other configs (run on the gpurun box)
# Usage: bash scripts/prof_cfg.sh TAG  -> gpurun_out/profcfg_TAG_{lv3b5,base8}/
set -o pipefail
TAG=${1:-p}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
WMI_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/profcfg_${TAG}_lv3b5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model large-v3 --beam 5 \
  --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/profcfg_${TAG}_lv3b5.log 2>&1 && \
WMI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/profcfg_${TAG}_base8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --clips-per-gpu 8 \
  --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/profcfg_${TAG}_base8.log 2>&1
echo "EXIT $?"
