"""Diagnostics for the persistent decoder: persist vs chain tokens, oracle margins."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
import synth  # noqa: E402
import wmi  # noqa: E402


def ctx_env(path, env, mc):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return wmi.WhisperContext.new(path, 0, max_clips=mc)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def toks(path, env, seeds, n=60):
    ctx = ctx_env(path, env, len(seeds))
    ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, s) for s in seeds])
    ctx.encode(1, 0)
    out = ctx.decode_greedy(n, suppress_eot=True)
    ctx.close()
    return out


mode = sys.argv[1] if len(sys.argv) > 1 else "all"
if mode in ("all", "trace"):
    path = synth.model_path("base")
    toks(path, {"WMI_PTRACE": "1"}, [40], 130)
if mode in ("all", "rows"):
    path = synth.model_path("base")
    P, C = {"WMI_PERSIST": "1"}, {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"}
    for seeds in ([40, 41], [41], [41, 40]):
        a, b = toks(path, P, seeds), toks(path, C, seeds)
        for i, s in enumerate(seeds):
            print("seeds", seeds, "clip seed", s, "persist", a[i][8:13], "chain", b[i][8:13],
                  "diff at", np.nonzero(a[i] != b[i])[0][:4], flush=True)
    import pyoracle
    om = pyoracle.OracleModel(path)
    mel = om.mel(synth.synth_pcm_f32(30.0, 41), n_threads=16)
    _, ck, cv = om.encode(mel, n_ctx=1500, n_threads=16)
    ref, margins = om.decode_greedy(ck, cv, 14, suppress_eot=True, n_threads=16)
    print("oracle seed 41", ref[8:13], "margins", np.round(margins[8:13], 5), flush=True)
