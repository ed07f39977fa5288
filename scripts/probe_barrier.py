#!/usr/bin/env python3
"""Grid-barrier probes on one GPU (wmi_bench_kernel 6-13): single-counter
barrier at 128/256/512 workgroups and the hierarchical (per-XCD group)
variants with and without agent-scope release/acquire fences."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

ctx = wmi.WhisperContext.new(synth.model_path("micro"), device=0, max_clips=1)
ctx.stage([synth.synth_pcm_f32(2.0, 1)])
ctx.run_staged(n_decode=4)
for k in range(6, 14):
    kb = ctx.bench_kernel(k, 20)
    print(f"probe {k}: {kb['name']}: {kb['avg_us']:.2f} us = {kb['avg_us'] / 32:.3f} us/barrier", flush=True)
ctx.close()
