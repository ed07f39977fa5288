#!/usr/bin/env python3
"""Per-layer encoder error against the C restatement (oracle/): the residual
stream after k layers on the GPU (WMI_ENC_LAYERS=k, wmi_debug_read 12) vs the
oracle's probe after layer k in ggml's AVX2 summation order (ref) and with
exact double dot products (exact).  Prints, per k: max |gpu - ref|, max
|gpu - exact| and the floor max |ref - exact|.  Usage: enc_layer_err.py MODEL"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
import synth  # noqa: E402
import wmi  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "small"
path = synth.model_path(model)
pcm = synth.synth_pcm_f32(30.0, 5)
om = pyoracle.OracleModel(path)
mel = om.mel(pcm, n_threads=16)
_, _, _, pr_ref = om.encode(mel, n_ctx=1500, n_threads=16, probe=True)
pyoracle.set_dot_mode(True)
_, _, _, pr_ex = om.encode(mel, n_ctx=1500, n_threads=16, probe=True)
pyoracle.set_dot_mode(False)
L = om.hp["n_audio_layer"]
n = om.hp["n_audio_state"]
for k in range(L + 1):
    os.environ["WMI_ENC_LAYERS"] = str(k)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    ctx.pcm_to_mel_batch([pcm])
    ctx.encode(1, 0)
    h = np.frombuffer(ctx.debug_read(12, 1500 * n * 4), np.float32).reshape(1500, n)
    ctx.close()
    print(f"{model} layer {k:2d}: |gpu-ref| {np.abs(h - pr_ref[k]).max():.3e}  |gpu-exact| {np.abs(h - pr_ex[k]).max():.3e}"
          f"  floor |ref-exact| {np.abs(pr_ref[k] - pr_ex[k]).max():.3e}  (mean {np.abs(h - pr_ref[k]).mean():.2e} /"
          f" {np.abs(h - pr_ex[k]).mean():.2e} / {np.abs(pr_ref[k] - pr_ex[k]).mean():.2e})", flush=True)
om.close()
