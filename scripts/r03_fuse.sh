#!/bin/bash
# fused one-row decoder: parity tests, phase traces, A/B against WMI_FUSE=0
set -o pipefail
TAG=${1:-f1}
O=gpurun_out
mkdir -p $O
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "fused_matches_unfused or persistent_matches_chain or greedy_tokens_micro or teacher_forced or batch_equals or logits_full" \
  > $O/fuse_t_$TAG.log 2>&1; rc=$?; tail -3 $O/fuse_t_$TAG.log; [ $rc -eq 0 ] || exit 1
WMI_PTRACE=1 timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > $O/fuse_trace_$TAG.log 2>&1 || exit 1
WMI_FUSE=0 WMI_PTRACE=1 timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > $O/nofuse_trace_$TAG.log 2>&1 || exit 1
bash scripts/ab.sh "WMI_FUSE=1" "WMI_FUSE=0" "WMI_FUSE=1" "WMI_FUSE=0" || exit 1
MODEL=small bash scripts/ab.sh "WMI_FUSE=1" "WMI_FUSE=0" || exit 1
MODEL=tiny bash scripts/ab.sh "WMI_FUSE=1" "WMI_FUSE=0" || exit 1
