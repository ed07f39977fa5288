#!/bin/bash
# One GPU session on the gpurun box (run from the repo root): the named steps
# in order, each under its own time limit; the first failing step ends the
# session (nothing more runs on the GPU after a fault, abort or time limit).
#
#   bash scripts/session.sh TAG STEP [STEP ...]
#
# steps (outputs under gpurun_out/, prefixed TAG):
#   tests[=K]          pytest -m gpu (optionally -k K): TAG_tests.log
#   smoke              __graft_entry__.smoke(): TAG_smoke.log
#   bench[=ARGS]       bench.py ARGS (default: the driver's line, all configs + CPU baseline): TAG_bench.json
#   trace=MODEL:ROWS   decoder phase trace (WMI_PTRACE) of a greedy run: TAG_trace_MODEL_ROWS.log
#   beamtrace=MODEL:K  the same for a K-beam search (16 steps): TAG_beamtrace_MODEL_K.log
#   prof               rocprofv3 kernel-trace summary of the base bench: TAG_prof/
#   pmc=MODEL:CLIPS    FETCH_SIZE / WRITE_SIZE passes of the persistent decoder (kernel 14): TAG_pmc_MODEL_CLIPS*
#   encpmc=MODEL:CLIPS per-kernel MFMA utilisation of the encoder: TAG_encpmc_MODEL_CLIPS.txt
#   gemmab=MODEL:CLIPS one-clip encoder GEMM paths A/B (scripts/gemm_p_ab.py): TAG_gemmab_MODEL_CLIPS.log
#   probe=MODEL:CLIPS:NTOK[:beam]  step-logit parity probe (scripts/parity_probe.py): TAG_probe_MODEL_CLIPS.log
#   ab=ENV1,ENV2,...   bench (base, 1 clip, 10 steps) alternating environments, e.g. ab=WMI_LIB=whisper.rs_amd/ab/X/libwhisper_mi355x.so,WMI_LIB=
#                      (MODEL, CPG, BEAM in the environment select another config): TAG_ab.txt
# Replaces the one-off drivers of rounds 1-3 (their evidence is under profiles/).
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
export WMI_MODEL_CACHE=/tmp/wmi_models
O=$R/gpurun_out/$TAG
for step in "$@"; do
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  echo "[session] $step"
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 1100 python3 -u -m pytest -x -v -s --durations=40 --timeout 700 --timeout-method thread tests/ -m gpu "${k[@]}" \
        > ${O}_tests.log 2>&1; rc=$?
      grep -E "passed|failed|compared over|error" ${O}_tests.log | tail -n 4
      [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || exit 1
      tail -n 1 ${O}_smoke.log ;;
    bench)
      timeout -k 10 800 python3 bench.py $arg > ${O}_bench.json 2> ${O}_bench.err || exit 1
      python3 -c "
import json; d=json.load(open('${O}_bench.json')); print('bench', d['value'], d['stage_ms'], (d.get('roofline') or {}).get('frac'))
[print(' ', k, v.get('audio_s_per_s'), v.get('decode_ms'), v.get('encoder_ms'), (v.get('roofline') or {}).get('frac')) for k, v in d.get('configs', {}).items()]" ;;
    beamtrace)
      m=${arg%%:*}; k=${arg#*:}
      timeout -k 10 400 python3 -u scripts/diag_persist.py beamtrace $m $k 16 > ${O}_beamtrace_${m}_${k}.log 2>&1 || exit 1
      grep "wg 0: step" ${O}_beamtrace_${m}_${k}.log ;;
    trace)
      m=${arg%%:*}; rows=${arg#*:}
      timeout -k 10 400 python3 -u scripts/diag_persist.py trace $m $rows > ${O}_trace_${m}_${rows}.log 2>&1 || exit 1
      grep "wg 0: step" ${O}_trace_${m}_${rows}.log ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && WMI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d ${O}_prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --configs none \
        --no-cpu-baseline > ${O}_prof.log 2>&1) || exit 1
      head -n 4 ${O}_prof/run_kernel_stats.csv ;;
    pmc)
      m=${arg%%:*}; c=${arg#*:}
      export WMI_NO_GRAPH=1
      timeout -k 10 300 python3 scripts/kernel_probe.py $m 14 1 128 $c > ${O}_pmc_${m}_${c}_warm.log 2>&1 || exit 1
      (cd /tmp && export TMPDIR=/tmp && \
        timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${O}_pmc_${m}_${c}_fetch -o run -- \
          python3 $R/scripts/kernel_probe.py $m 14 3 128 $c > ${O}_pmc_${m}_${c}_fetch.log 2>&1 && \
        timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d ${O}_pmc_${m}_${c}_write -o run -- \
          python3 $R/scripts/kernel_probe.py $m 14 3 128 $c > ${O}_pmc_${m}_${c}_write.log 2>&1 && \
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_pmc_${m}_${c}_trace -o run -- \
          python3 $R/scripts/kernel_probe.py $m 14 3 128 $c > ${O}_pmc_${m}_${c}_trace.log 2>&1) || exit 1
      unset WMI_NO_GRAPH
      cat ${O}_pmc_${m}_${c}_trace.log ;;
    encpmc)
      # per-kernel MFMA utilisation of the encoder: a kernel-trace pass and a
      # SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass over the same encodes
      m=${arg%%:*}; c=${arg#*:}
      (cd /tmp && export TMPDIR=/tmp && \
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_encpmc_${m}_${c}_trace -o run -- \
          python3 $R/scripts/encode_probe.py $m $c 5 > ${O}_encpmc_${m}_${c}_trace.log 2>&1 && \
        timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
          -d ${O}_encpmc_${m}_${c}_pmc -o run -- python3 $R/scripts/encode_probe.py $m $c 5 \
          > ${O}_encpmc_${m}_${c}_pmc.log 2>&1) || exit 1
      python3 scripts/enc_mfma_summary.py ${O}_encpmc_${m}_${c}_trace ${O}_encpmc_${m}_${c}_pmc ${O}_encpmc_${m}_${c}.txt ;;
    gemmab)
      # one-clip encoder GEMM paths (WMI_GEMM_P 0 / 1 / 2): bitwise check + interleaved encode medians
      m=${arg%%:*}; c=${arg#*:}
      timeout -k 10 300 python3 -u scripts/gemm_p_ab.py $m $c 3 20 > ${O}_gemmab_${m}_${c}.log 2>&1 || exit 1
      tail -n 3 ${O}_gemmab_${m}_${c}.log ;;
    probe)
      IFS=: read -ra pa <<< "$arg"
      timeout -k 10 600 python3 -u scripts/parity_probe.py "${pa[@]}" > ${O}_probe_${pa[0]}_${pa[1]}${pa[3]}.log 2>&1 || exit 1
      grep "\[probe\]" ${O}_probe_${pa[0]}_${pa[1]}${pa[3]}.log | tail -n 12 ;;
    ab)
      IFS=, read -ra envs <<< "$arg"
      for rep in 1 2; do
        for e in "${envs[@]}"; do
          timeout -k 10 300 env $e python3 bench.py --model ${MODEL:-base} --beam ${BEAM:-0} --clips-per-gpu ${CPG:-1} \
            --steps ${STEPS:-10} --warmup 2 --configs none --no-cpu-baseline 2>/dev/null > ${O}_ab_one.json || exit 1
          python3 -c "
import json; d=json.load(open('${O}_ab_one.json')); print('$e', d['value'], d['stage_ms']['decode_ms'], d['encoder_ms'], d['stage_ms']['mel_ms'])" \
            | tee -a ${O}_ab.txt
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[session] EXIT 0"
