"""Bitwise comparison of two builds of the library (scripts/build_variant.sh)
on the encoder output and the persistent decoder: greedy ids and last-step
logits of base (1 clip and 8 clips), micro and small.  Usage: lib_equal.py LIB_A LIB_B (run on the gpurun box)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = (("base", 1, 1500, 30.0), ("base", 8, 1500, 30.0), ("micro", 3, 64, 2.0), ("small", 1, 1500, 30.0))


def run_one(out):
    sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
    import synth
    import wmi
    res = {}
    for model, nc, ctx_n, secs in CASES:
        os.environ["WMI_PERSIST_LOGITS"] = "1"
        ctx = wmi.WhisperContext.new(synth.model_path(model), 0, max_clips=nc)
        ctx.set_audio_ctx(ctx_n)
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(secs, 1234 + i) for i in range(nc)])
        ctx.encode(1, 0)
        res[f"{model}_{nc}_enc"] = np.stack([ctx.encoder_out(i) for i in range(nc)])
        for i in range(nc):
            k, v = ctx.cross_kv(i)
            res[f"{model}_{nc}_ck{i}"] = k
            res[f"{model}_{nc}_cv{i}"] = v
        toks = np.stack(ctx.decode_greedy(48, suppress_eot=True))
        V = ctx.hparams["n_vocab"]
        lg = np.frombuffer(ctx.debug_read(2, nc * V * 4), np.float32).copy()
        ctx.close()
        res[f"{model}_{nc}_tok"] = toks
        res[f"{model}_{nc}_lg"] = lg
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        sys.exit(0)
    outs = []
    for i, lib in enumerate(sys.argv[1:3]):
        o = f"/tmp/lib_equal_{i}.npz"
        env = dict(os.environ, WMI_LIB=os.path.abspath(lib), WMI_MODEL_CACHE=os.environ.get("WMI_MODEL_CACHE", "/tmp/wmi_models"))
        subprocess.run([sys.executable, os.path.abspath(__file__), "--one", o], env=env, check=True)
        outs.append(np.load(o))
    bad = 0
    for k in outs[0].files:
        same = np.array_equal(outs[0][k], outs[1][k])
        print(k, "bitwise equal" if same else f"DIFFER (max |d| {np.abs(outs[0][k].astype(np.float64) - outs[1][k]).max():.3g})")
        if not same:
            d = np.argwhere(outs[0][k] != outs[1][k])
            print(f"   {len(d)} of {outs[0][k].size} differ; first at {d[:4].tolist()}: "
                  f"{[outs[0][k][tuple(i)] for i in d[:4]]} vs {[outs[1][k][tuple(i)] for i in d[:4]]}")
        bad += not same
    print("LIB_EQUAL", "OK" if not bad else f"{bad} differ")
    sys.exit(1 if bad else 0)
