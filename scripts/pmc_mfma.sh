#!/bin/bash
# MFMA utilisation of the encoder kernels from rocprofv3 PMC counters:
# SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) and GRBM_GUI_ACTIVE
# (summed over the 8 XCDs), one pass per kernel (bench KERNELS ids 1 = mlp.0
# GEMM, 2 = encoder attention, 3 = cross-K/V GEMM).  Usage: bash scripts/pmc_mfma.sh TAG [model]
set -o pipefail
TAG=${1:-m}
MODEL=${2:-base}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
export WMI_NO_GRAPH=1
timeout -k 10 200 python3 $R/scripts/kernel_probe.py $MODEL 1 2 > $R/gpurun_out/mfma_${TAG}_warm.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for W in 1 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $R/gpurun_out/mfma_${TAG}_$W -o run -- python3 $R/scripts/kernel_probe.py $MODEL $W 20 \
    > $R/gpurun_out/mfma_${TAG}_$W.log 2>&1 || exit 1
done
echo "EXIT 0"
