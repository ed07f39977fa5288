"""Decoder logit parity probe (GPU box): every step's logits of the persistent
greedy decode (WMI_LOGITS_ALL=1) against the oracle teacher-forced on the
device's own ids, per instance; prints max |diff|, max |logit|, id agreement
and the number of distinct id sequences.  Measurement for the bars in
tests/test_gpu_parity.py (not a test itself).

  python3 scripts/parity_probe.py MODEL CLIPS N_TOK [beam]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
os.environ["WMI_LOGITS_ALL"] = "1"
import pyoracle  # noqa: E402
import synth  # noqa: E402
import wmi  # noqa: E402

model, clips, n_tok = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
beam = len(sys.argv) > 4 and sys.argv[4] == "beam"
thr = min(16, os.cpu_count() or 8)
path = synth.model_path(model)
om = pyoracle.OracleModel(path)
ctx = wmi.WhisperContext.new(path, 0, max_clips=clips)
pcm = [synth.synth_pcm_f32(30.0, 1234 + i) for i in range(clips)]
t0 = time.time()
refs = []
for p in pcm:
    _, ck, cv = om.encode(om.mel(p, n_threads=thr), n_ctx=1500, n_threads=thr)
    refs.append((ck, cv))
print(f"[probe] {model}: oracle encode {time.time() - t0:.1f}s", flush=True)
ctx.pcm_to_mel_batch(pcm)
ctx.encode(1, 0)
prompt = om.prompt()
np_ = len(prompt)
eot = om.special["eot"]
if beam:
    for i, (ck, cv) in enumerate(refs[:1]):
        ctx.pcm_to_mel_batch(pcm[i:i + 1])
        ctx.encode(1, 0)
        got, sc = ctx.decode_beam(5, n_tok, suppress_eot=True)[0]
        ref, rsc, gap, sg = om.decode_beam(ck, cv, 5, n_tok, suppress_eot=True, n_threads=thr, step_gaps=True)
        feed = np.array(prompt + list(got[:-1]), np.int32)
        lg = ctx.decode_logits(feed, 0)
        lr = om.decode_logits(ck, cv, feed, n_threads=thr)
        d = np.abs(lg - lr)
        print(f"[probe] beam clip {i}: ids equal {bool(np.array_equal(got, ref))} ({len(got)} vs {len(ref)}), "
              f"score {sc:.5f} vs {rsc:.5f}, min sel margin {gap:.2e}; teacher-forced best hyp: max|d| {d.max():.3e} "
              f"max|logit| {np.abs(lr).max():.2f}", flush=True)
    sys.exit(0)
t0 = time.time()
got = ctx.decode_greedy(n_tok, suppress_eot=True)
lg_all = ctx.step_logits(np_ + n_tok - 1)
print(f"[probe] gpu decode {time.time() - t0:.1f}s", flush=True)
seqs = set()
worst = 0.0
for i, (ck, cv) in enumerate(refs):
    g = got[i]
    seqs.add(tuple(int(x) for x in g))
    feed = np.array(prompt + list(g[:-1]), np.int32)
    lr = om.decode_logits(ck, cv, feed, n_threads=thr)[np_ - 1:]
    lgd = lg_all[np_ - 1:np_ - 1 + n_tok, i, :]
    d = np.abs(lgd - lr)
    worst = max(worst, float(d.max()))
    lrs = lr.copy()
    lrs[:, eot] = -np.inf
    top2 = np.sort(lrs, axis=1)[:, -2:]
    marg = top2[:, 1] - top2[:, 0]
    am = lrs.argmax(1)
    lgs = lgd.copy()
    lgs[:, eot] = -np.inf
    selfc = (lgs.argmax(1) == g).all()
    agree = (am == g) | (marg < 1e-3)
    ref_ids, _ = om.decode_greedy(ck, cv, n_tok, suppress_eot=True, n_threads=thr)
    dif = np.nonzero(ref_ids != g)[0]
    print(f"[probe] clip {i}: max|d| {d.max():.3e} (per-step max of mean {d.max(1).mean():.2e}) max|logit| "
          f"{np.abs(lr).max():.2f}; ids self-consistent {bool(selfc)}; oracle argmax agrees {int(agree.sum())}/{n_tok} "
          f"(decisive {int((marg >= 1e-3).sum())}); free-run equal to oracle for {dif[0] if dif.size else n_tok}",
          flush=True)
print(f"[probe] {model} x{clips}: worst {worst:.3e}; distinct id sequences {len(seqs)}", flush=True)
ctx.close()
om.close()
