#!/usr/bin/env python3
"""A/B of the one-clip encoder GEMM paths (WMI_GEMM_P = 0: k_gemm, 1:
k_gemm_p; the settings compared: GEMM_P_SETTINGS, default 0,1 — round 6
also measured settings 2-4, since removed: profiles/r06/gemm_p_ab.txt): the encoder
output and cross K / V must be bitwise equal across the settings; the encode
time is the median of `iters` encodes per round, the settings interleaved
over `rounds` rounds in one process.  Usage: gemm_p_ab.py [model] [clips]
[rounds] [iters]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "base"
clips = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
path = synth.model_path(model)
pcm = [synth.synth_pcm_f32(30.0, 1234 + i) for i in range(clips)]
settings = tuple(os.environ.get("GEMM_P_SETTINGS", "0,1").split(","))
VAR = os.environ.get("AB_VAR", "WMI_GEMM_P")  # the knob compared (WMI_GELU_CALC: the GELU epilogues)
ctxs = {}
for g in settings:
    os.environ[VAR] = g
    ctxs[g] = wmi.WhisperContext.new(path, device=0, max_clips=clips)
    ctxs[g].pcm_to_mel_batch(pcm)
del os.environ[VAR]
ref = None
for g in settings:
    ctx = ctxs[g]
    ctx.encode(1, 0)
    got = [(ctx.encoder_out(i), *ctx.cross_kv(i)) for i in range(clips)]
    if ref is None:
        ref = got
    else:
        same = all(np.array_equal(x, y) for a, b in zip(ref, got) for x, y in zip(a, b))
        print(f"{VAR}={g}: bitwise equal to {VAR}={settings[0]}: {same}", flush=True)
        if not same:
            sys.exit(1)
times = {g: [] for g in settings}
for r in range(rounds):
    for g in settings:
        ctx = ctxs[g]
        for _ in range(3):
            ctx.encode(1, 0)
        t = []
        for _ in range(iters):
            ctx.encode(1, 0)
            t.append(ctx.timings()["encode_ms"])
        times[g].append(float(np.median(t)))
    print(f"round {r}: " + ", ".join(f"{VAR}={g} {times[g][-1]:.4f} ms" for g in settings), flush=True)
for g in settings:
    print(f"{model} x{clips} {VAR}={g}: encode median over rounds {np.median(times[g]):.4f} ms "
          f"(rounds {', '.join(f'{x:.4f}' for x in times[g])})", flush=True)
for c in ctxs.values():
    c.close()
