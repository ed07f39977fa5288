#!/usr/bin/env python3
"""Print the timestamp-decoding output of the micro model (debug aid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd")]
import synth, wmi  # noqa
ctx = wmi.WhisperContext.new(synth.model_path(sys.argv[1] if len(sys.argv) > 1 else "micro"), 0, max_clips=1)
if len(sys.argv) < 2:
    ctx.set_audio_ctx(64)
pcm = synth.synth_pcm_f32(float(sys.argv[2]) if len(sys.argv) > 2 else 4.0, 21)
ctx.pcm_to_mel_batch([pcm]); ctx.encode(1, 0)
sp = ctx.special
w = ctx.decode_timestamps([sp["sot"]] + ([sp["sot"] + 1, sp["transcribe"]] if sp["multilingual"] else []), 24)
print("window:", [(t["id"] - sp["beg"] if t["id"] > sp["beg"] else t["id"], round(t["p"], 4)) for t in w])
segs = ctx.transcribe(pcm, max_tokens=24)
print("segments:", len(segs))
for s in segs[:10]:
    print(s["t0"], s["t1"], s["text"][:60], len(s["tokens"]))
ctx.close()
