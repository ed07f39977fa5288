#!/bin/bash
# A/B of library variants on the gpurun box: for each NAME, the decoder phase
# trace (WMI_PTRACE, base, one clip) and bench.py (base, no extra configs).
# NAME "main" is the in-tree library.  Usage: bash scripts/ab_lib.sh TAG NAME...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
for v in "$@"; do
  if [ "$v" = main ]; then unset WMI_LIB; else export WMI_LIB=$PWD/whisper.rs_amd/ab/$v/libwhisper_mi355x.so; fi
  timeout -k 10 200 python3 -u scripts/diag_persist.py trace base 1 > gpurun_out/ab_${TAG}_${v}_trace.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --configs none --no-cpu-baseline \
    > gpurun_out/ab_${TAG}_${v}.json 2> gpurun_out/ab_${TAG}_${v}.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_${TAG}_${v}.json'))
print('$v', d['value'], d['stage_ms']['decode_ms'], d['encoder_ms'], d['roofline']['avg_us'])"
  grep "wg 0: step" gpurun_out/ab_${TAG}_${v}_trace.log
done
echo "AB EXIT 0"
