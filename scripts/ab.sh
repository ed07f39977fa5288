#!/bin/bash
# A/B timing of decoder variants on the gpurun box: bench.py base, 3 steps
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['stage_ms']['decode_ms'], d['roofline']['avg_us'])"; }
run WMI_X=0 && run WMI_NO_FUSE=1 && run WMI_LIB=$PWD/whisper.rs_amd/libwhisper_mi355x_nt.so && \
run WMI_LIB=$PWD/whisper.rs_amd/libwhisper_mi355x_nt.so WMI_NO_FUSE=1
