"""Diagnostic (not collected by pytest): print GPU-vs-oracle error magnitudes."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
import synth, pyoracle, wmi

def f16(b): return np.asarray(b, np.uint16).view(np.float16).astype(np.float32)

def run(model, n_ctx, secs=30.0, ndec=16):
    path = synth.model_path(model)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    pcm = synth.synth_pcm_f32(secs, 1234)
    t = time.time(); mel = om.mel(pcm, 16); enc_r, ck_r, cv_r, pr = om.encode(mel, n_ctx=n_ctx, n_threads=16, probe=True); tcpu = time.time() - t
    ctx.set_audio_ctx(n_ctx); ctx.pcm_to_mel_batch([pcm]); ctx.encode(1, 0)
    enc = ctx.encoder_out(0); ck, cv = ctx.cross_kv(0)
    print(f"[{model} n_ctx={n_ctx}] cpu {tcpu:.2f}s  mel maxdiff {np.abs(ctx.mel(0)-mel).max():.2e}")
    print(f"  enc maxabs {np.abs(enc-enc_r).max():.3e} meanabs {np.abs(enc-enc_r).mean():.3e} |enc|max {np.abs(enc_r).max():.2f}")
    print(f"  ck maxabs {np.abs(f16(ck)-f16(ck_r)).max():.3e} cv maxabs {np.abs(f16(cv)-f16(cv_r)).max():.3e}  exact ck {(ck==ck_r).mean():.4f}")
    t = time.time(); ref, mg = om.decode_greedy(ck_r, cv_r, ndec, suppress_eot=True, n_threads=16); tdec = time.time() - t
    got = ctx.decode_greedy(ndec, suppress_eot=True)[0]
    print(f"  greedy oracle {ref.tolist()}\n  greedy gpu    {got.tolist()}\n  min margin {mg.min():.3e} cpu dec {tdec:.2f}s")
    toks = np.array(om.prompt() + ref[:6].tolist(), np.int32)
    lr = om.decode_logits(ck_r, cv_r, toks, 16); lg = ctx.decode_logits(toks, 0)
    print(f"  logits maxabs {np.abs(lr-lg).max():.3e} |logit|max {np.abs(lr).max():.2f}")
    ctx.close(); om.close()

if __name__ == "__main__":
    for spec in sys.argv[1:]:
        m, c = spec.split(":")
        run(m, int(c))
