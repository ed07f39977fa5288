#!/bin/bash
# HBM traffic of the bench's roofline kernel from rocprofv3 PMC counters
# (MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE in separate passes,
# kernel trace in a third).  Decoder kernels launch eagerly (WMI_NO_GRAPH).
# Usage (repo root on the gpurun box): bash scripts/pmc_pass.sh TAG [model] [kernel-id] [iters] [n_decode]
set -o pipefail
TAG=${1:-p}
MODEL=${2:-base}
WHICH=${3:-0}
IT=${4:-20}
ND=${5:-8}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
export WMI_NO_GRAPH=1
timeout -k 10 200 python3 $R/scripts/kernel_probe.py $MODEL $WHICH 2 $ND > $R/gpurun_out/pmc_${TAG}_warm.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_${TAG}_fetch -o run -- \
  python3 $R/scripts/kernel_probe.py $MODEL $WHICH $IT $ND > $R/gpurun_out/pmc_${TAG}_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_${TAG}_write -o run -- \
  python3 $R/scripts/kernel_probe.py $MODEL $WHICH $IT $ND > $R/gpurun_out/pmc_${TAG}_write.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_${TAG}_trace -o run -- \
  python3 $R/scripts/kernel_probe.py $MODEL $WHICH $IT $ND > $R/gpurun_out/pmc_${TAG}_trace.log 2>&1
echo "EXIT $?"
