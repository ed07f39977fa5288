#!/usr/bin/env python3
"""Beam-search decode time, persistent decoder vs kernel chain (WMI_PERSIST).
Usage: beam_probe.py [model] [beam] [n_tok]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n_tok = int(sys.argv[3]) if len(sys.argv) > 3 else 32
path = synth.model_path(model)
pcm = synth.synth_pcm_f32(30.0, 1234)
for flag in ("1", "0"):
    os.environ["WMI_PERSIST"] = flag
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    ctx.pcm_to_mel_batch([pcm])
    ctx.encode(1, 0)
    ctx.decode_beam(K, 4, suppress_eot=True)
    t0 = time.perf_counter()
    toks, score = ctx.decode_beam(K, n_tok, suppress_eot=True)[0]
    dt = time.perf_counter() - t0
    print(f"WMI_PERSIST={flag}: {model} x {K} beams, {n_tok} tokens: {dt * 1e3:.1f} ms "
          f"({dt * 1e3 / (n_tok + 3):.2f} ms/step), score {score:.4f}, ids {list(toks[:8])}", flush=True)
    ctx.close()
