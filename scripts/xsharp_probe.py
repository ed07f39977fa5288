"""Design probe for the audio-dependent "-xsharp" synthetic models (CPU, oracle
only): per tone clip the oracle's greedy ids (distinct sequences, decisive
steps) and its 5-beam selection margins.  Usage:
  python scripts/xsharp_probe.py large-v3 conv1=20,pe=3,te=1 --clips 8 --tok 64 --beam 40
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
import synth  # noqa: E402


def hook_for(spec):
    sc = dict(conv1=1.0, pe=1.0, te=1.0, lnw=1.0, co=1.0)
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        sc[k] = float(v)

    def hook(name, arr):
        s = {"encoder.conv1.weight": sc["conv1"], "decoder.positional_embedding": sc["pe"],
             "decoder.token_embedding.weight": sc["te"], "decoder.ln.weight": sc["lnw"]}.get(name)
        if name.startswith("decoder.blocks.") and name.endswith("cross_attn.out.weight"):
            s = sc["co"]
        return arr if s is None or s == 1.0 else (arr.astype(np.float32) * s).astype(arr.dtype)
    return hook


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("spec")
    ap.add_argument("--clips", type=int, default=8)
    ap.add_argument("--tok", type=int, default=64)
    ap.add_argument("--beam", type=int, default=0)
    ap.add_argument("--beam-seeds", type=int, default=4)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seed0", type=int, default=1234)
    a = ap.parse_args()
    path = f"/tmp/wmi_models/x-{a.model}-{a.spec.replace(',', '_').replace('=', '')}.bin"
    if not os.path.exists(path):
        t0 = time.time()
        synth.write_ggml(path, a.model, tensor_hook=hook_for(a.spec))
        print(f"wrote {path} in {time.time() - t0:.1f} s", flush=True)
    om = pyoracle.OracleModel(path)
    seqs = []
    for i in range(a.clips):
        sd = a.seed0 + i
        t0 = time.time()
        pcm = synth.synth_pcm_tones(30.0, sd)
        _, ck, cv = om.encode(om.mel(pcm, n_threads=a.threads), n_ctx=1500, n_threads=a.threads)
        t1 = time.time()
        ids, m = om.decode_greedy(ck, cv, a.tok, suppress_eot=True, n_threads=a.threads)
        t2 = time.time()
        seqs.append(tuple(ids))
        line = (f"seed {sd}: encode {t1 - t0:.1f} s greedy {t2 - t1:.1f} s; decisive {(m >= 1e-3).sum()}/{a.tok}, "
                f"min margin {m.min():.2e}, distinct ids {len(set(ids))}, first {list(ids[:8])}")
        if a.beam and i < a.beam_seeds:
            _, _, gap, sg = om.decode_beam(ck, cv, 5, a.beam, suppress_eot=True, n_threads=a.threads, step_gaps=True)
            first = int(np.argmax(sg < 2e-3)) if (sg < 2e-3).any() else a.beam
            line += f"; beam5 first near-tie step {first} (final gap {gap:.2e}) beam {time.time() - t2:.1f} s"
        print(line, flush=True)
    print(f"{len(set(seqs))} distinct sequences over {a.clips} clips")


if __name__ == "__main__":
    main()
