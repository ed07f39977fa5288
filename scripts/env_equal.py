"""Bitwise comparison of two environment settings of the library on the
encoder outputs (ln_post, cross K/V) and the greedy decode (ids, last-step
logits).  Usage: env_equal.py "ENV_A=1" "ENV_B=0" (run on the gpurun box)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = (("base", 8), ("base", 1), ("small", 8), ("tiny", 3))


def run_one(out):
    sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
    import synth
    import wmi
    res = {}
    os.environ["WMI_PERSIST_LOGITS"] = "1"
    for model, nc in CASES:
        ctx = wmi.WhisperContext.new(synth.model_path(model), 0, max_clips=nc)
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, 1234 + i) for i in range(nc)])
        ctx.encode(1, 0)
        for i in range(nc):
            res[f"{model}_{nc}_enc{i}"] = ctx.encoder_out(i)
            k, v = ctx.cross_kv(i)
            res[f"{model}_{nc}_ck{i}"] = k
            res[f"{model}_{nc}_cv{i}"] = v
        toks = np.stack(ctx.decode_greedy(24, suppress_eot=True))
        V = ctx.hparams["n_vocab"]
        res[f"{model}_{nc}_tok"] = toks
        res[f"{model}_{nc}_lg"] = np.frombuffer(ctx.debug_read(2, nc * V * 4), np.float32).copy()
        ctx.close()
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        sys.exit(0)
    outs = []
    for i, spec in enumerate(sys.argv[1:3]):
        o = f"/tmp/env_equal_{i}.npz"
        env = dict(os.environ)
        for kv in spec.split(","):
            if kv:
                k, v = kv.split("=", 1)
                env[k] = v
        subprocess.run([sys.executable, os.path.abspath(__file__), "--one", o], env=env, check=True)
        outs.append(np.load(o))
    bad = 0
    for k in outs[0].files:
        same = np.array_equal(outs[0][k], outs[1][k])
        if not same:
            print(k, f"DIFFER (max |d| {np.abs(outs[0][k].astype(np.float64) - outs[1][k]).max():.3g})")
            d = np.argwhere(outs[0][k] != outs[1][k])
            print(f"   {len(d)} of {outs[0][k].size} differ; first at {d[:4].tolist()}: "
                  f"{[outs[0][k][tuple(i)] for i in d[:4]]} vs {[outs[1][k][tuple(i)] for i in d[:4]]}")
        bad += not same
    print("ENV_EQUAL", "OK" if not bad else f"{bad} of {len(outs[0].files)} differ", f"({len(outs[0].files)} arrays)")
    sys.exit(1 if bad else 0)
