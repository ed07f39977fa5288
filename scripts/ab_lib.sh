#!/bin/bash
# A/B of library variants on the gpurun box: for each variant, the decoder
# phase trace (WMI_PTRACE, base, one clip) and bench.py (base, no extra
# configs).  A variant is "main" (the in-tree library), NAME (the library
# built by scripts/build_variant.sh NAME) or "env:VAR=VAL[,VAR=VAL]" (the
# in-tree library under those environment variables).
# Usage: bash scripts/ab_lib.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
for v in "$@"; do
  unset WMI_LIB
  envs=""
  case "$v" in
    main) ;;
    env:*) envs=$(echo "${v#env:}" | tr ',' ' ');;
    *) export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so;;
  esac
  n=$(echo "$v" | tr ':=,' '___')
  timeout -k 10 200 env $envs python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/ab_${TAG}_${n}_trace.log 2>&1 || exit 1
  timeout -k 10 200 env $envs python3 bench.py --steps 10 --warmup 2 --configs none --no-cpu-baseline \
    > gpurun_out/ab_${TAG}_${n}.json 2> gpurun_out/ab_${TAG}_${n}.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_${TAG}_${n}.json'))
print('$v', d['value'], d['stage_ms']['decode_ms'], d['encoder_ms'], d['roofline']['avg_us'])"
  grep "wg 0: step" gpurun_out/ab_${TAG}_${n}_trace.log
done
echo "AB EXIT 0"
