#!/usr/bin/env python3
"""Short driver for rocprofv3 --pmc passes: one staged pipeline (8 decode
tokens) then `iters` back-to-back launches of one bench kernel (bench.py's
KERNELS ids: 0 = decoder logits GEMV).  Usage: kernel_probe.py [model] [which] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "base"
which = int(sys.argv[2]) if len(sys.argv) > 2 else 0
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ctx = wmi.WhisperContext.new(synth.model_path(model), device=0, max_clips=1)
ctx.stage([synth.synth_pcm_f32(30.0, 1234)])
ctx.run_staged(n_decode=8)
kb = ctx.bench_kernel(which, iters)
print(f"{kb['name']}: {kb['avg_us']:.2f} us, alg bytes {kb['alg_bytes']:.0f}", flush=True)
ctx.close()
