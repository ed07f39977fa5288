#!/bin/bash
# PMC passes over the encoder attention kernel (bench id 2) at one base clip,
# plus a kernel-trace of a short bench, for the enc3 / enc4 investigation.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 200 python3 $R/scripts/kernel_probe.py base 2 2 > $O/pa_warm.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
for v in 3 4; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    WMI_ENC_ATTN=$v WMI_ENC_ATTN_NW=${NW:-4} timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pa_v${v}_p$i -o run -- \
      python3 $R/scripts/kernel_probe.py base 2 10 > $O/pa_v${v}_p$i.log 2>&1 || exit 1
  done
done
cd $R
WMI_ENC_ATTN=4 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pa_trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pa_trace.log 2>&1 || exit 1
echo "EXIT 0"
