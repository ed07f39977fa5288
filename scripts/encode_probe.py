#!/usr/bin/env python3
"""rocprofv3 driver for the encoder: mel once, then `iters` encodes of the
same clips (conv stem -> encoder blocks -> ln_post -> cross K/V), so every
encoder kernel appears iters times.  Usage: encode_probe.py [model] [clips] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "base"
clips = int(sys.argv[2]) if len(sys.argv) > 2 else 1
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = wmi.WhisperContext.new(synth.model_path(model), device=0, max_clips=clips)
ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, 1234 + i) for i in range(clips)])
for _ in range(iters):
    ctx.encode(1, 0)
print(f"encode_probe {model} x{clips}: {iters} encodes, last {ctx.timings()['encode_ms']:.3f} ms", flush=True)
ctx.close()
