#!/usr/bin/env python3
"""Short driver for rocprofv3 --pmc passes: one staged pipeline (8 decode
tokens, or n_decode) then `iters` back-to-back launches of one bench kernel
(wmi_bench_kernel ids: 14 = the persistent greedy decoder over n_decode tokens,
0 = the chain's logits GEMV).  Usage: kernel_probe.py [model] [which] [iters] [n_decode] [clips]
(clips > 1: that many staged clips decode as rows of one multi-row launch)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "base"
which = int(sys.argv[2]) if len(sys.argv) > 2 else 0
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
n_decode = int(sys.argv[4]) if len(sys.argv) > 4 else 8
clips = int(sys.argv[5]) if len(sys.argv) > 5 else 1
ctx = wmi.WhisperContext.new(synth.model_path(model), device=0, max_clips=clips)
ctx.stage([synth.synth_pcm_f32(30.0, 1234 + i) for i in range(clips)])
ctx.run_staged(n_decode=n_decode)
kb = ctx.bench_kernel(which, iters)
print(f"{kb['name']}: {kb['avg_us']:.2f} us, alg bytes {kb['alg_bytes']:.0f}", flush=True)
ctx.close()
