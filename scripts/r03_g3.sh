#!/bin/bash
set -o pipefail
# focused tests, decoder A/B, the full GPU suite, then the kernel table of two
# large-v3 x 5-beam bench steps (configs[4])
TAG=${1:-r03f}
mkdir -p gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "lds_kv or exp_matches or teacher or greedy or persistent_matches" > gpurun_out/t1_$TAG.log 2>&1 && echo TEST1_OK && \
bash scripts/ab_lib.sh $TAG main env:WMI_KVL=0 && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_$TAG.log 2>&1 && echo TEST_OK && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof_lv3b5_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model large-v3 --beam 5 \
  --steps 2 --warmup 1 --configs none --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_lv3b5_$TAG.log 2>&1 && echo PROF_OK && \
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python3 -u scripts/enc_layer_err.py small > gpurun_out/enc_layers_small_$TAG.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/enc_layer_err.py small-q5_1 > gpurun_out/enc_layers_smallq5_$TAG.log 2>&1 && echo ENC_OK
