#!/usr/bin/env python3
"""Dump the encoder output and cross K / V of fixed synthetic clips (tiny,
base, small at one clip; base at 8 clips) from the library WMI_LIB selects,
for bitwise comparisons of two builds:
    WMI_LIB=a.so enc_dump.py A.npz; WMI_LIB=b.so enc_dump.py B.npz; enc_dump.py --cmp A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    assert sorted(a.files) == sorted(b.files), (a.files, b.files)
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print(f"enc_dump cmp: {len(a.files)} arrays, {len(bad)} differ {bad[:8]}")
    sys.exit(1 if bad else 0)

import synth  # noqa: E402
import wmi  # noqa: E402

out = {}
for model, nc in (("tiny", 1), ("base", 1), ("small", 1), ("base", 8)):
    ctx = wmi.WhisperContext.new(synth.model_path(model), device=0, max_clips=nc)
    try:
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, 2100 + i) for i in range(nc)])
        ctx.encode(1, 0)
        for i in range(nc):
            k, v = ctx.cross_kv(i)
            out[f"{model}_{nc}_{i}_enc"] = ctx.encoder_out(i)
            out[f"{model}_{nc}_{i}_k"] = k
            out[f"{model}_{nc}_{i}_v"] = v
    finally:
        ctx.close()
np.savez(sys.argv[1], **out)
print(f"enc_dump: {len(out)} arrays -> {sys.argv[1]}")
