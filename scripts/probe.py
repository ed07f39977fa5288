#!/usr/bin/env python3
"""Decoder-step timeline (WMI_TRACE=1) and launch/barrier probes on one GPU.
Usage: WMI_TRACE=1 python3 scripts/probe.py [model] [n_decode]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "base"
n_dec = int(sys.argv[2]) if len(sys.argv) > 2 else 128
beam = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ctx = wmi.WhisperContext.new(synth.model_path(model), device=0, max_clips=1)
ctx.stage([synth.synth_pcm_f32(30.0, 1234)])
for i in range(2):
    t0 = time.perf_counter()
    ctx.run_staged(n_decode=n_dec, beam_size=beam)
    print(f"run {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms  {ctx.timings()}", flush=True)
for k in (4, 5, 6, 7, 8):
    kb = ctx.bench_kernel(k, 20)
    print(f"probe {k}: {kb['name']}: {kb['avg_us']:.2f} us", flush=True)
ctx.close()
