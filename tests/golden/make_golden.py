#!/usr/bin/env python3
"""Golden vectors for the CPU oracle, from an INDEPENDENT NumPy restatement.

The reference (szuwgh/whisper.rs) cannot run in this container and its own
tests pin no numbers, so parity with it is "unpinned".
What this script provides instead: a second, independent restatement of the
same path — written in NumPy, float64 accumulation, numpy FFT, f16 rounding
points emulated with np.float16 casts — whose outputs are committed as
fixtures.  tests/test_oracle.py requires the C oracle (oracle/wmi_oracle.c,
ggml-style f32 accumulation, reference FFT) to agree with them within the
tolerances written there; two implementations that share no code agreeing is
the pin the oracle gets.

Restated items (file:line into /root/reference/src/main.rs):
  mel      log_mel_spectrogram / clamp_and_normalize   :1554-1671
  window   whisper_encode mel copy                     :1816-1833
  encoder  conv stem, blocks, ln_post                  :1834-1986 (ggml-1.0.3 op semantics)
  crossKV  Kc = f16((Wk E) * (n/h)^-0.25), Vc          :1990-2060
  decoder  SURVEY §A.7 (absent from the reference)

Run:  python tests/golden/make_golden.py   (writes tests/golden/micro_golden.npz)
      python tests/golden/make_golden.py --f32   (micro_f32_golden.npz: the
      same model as an f32 / ftype-0 file, whose matmuls round nothing)
"""
from __future__ import annotations

import hashlib
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))
import synth  # noqa: E402

N_CTX = 64          # exp_n_audio_ctx used for the fixture (2 * 64 = 128 mel frames)
SECONDS = 2.0
SEED = 1234
N_GREEDY = 12


def read_ggml(path):
    with open(path, "rb") as f:
        data = f.read()
    off = 0

    def take(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, data, off)
        off += struct.calcsize(fmt)
        return v

    (magic,) = take("<I")
    assert magic == 0x67676D6C
    hp = dict(zip(synth.HPARAM_ORDER, take("<11i")))
    n_mel, n_ff = take("<ii")
    filters = np.frombuffer(data, "<f4", n_mel * n_ff, off).reshape(n_mel, n_ff).astype(np.float64)
    off += 4 * n_mel * n_ff
    (nv,) = take("<i")
    for _ in range(nv):
        (ln,) = take("<I")
        off += ln
    tensors = {}
    while len(data) - off >= 12:
        n_dims, ln, ftype = take("<iii")
        ne = take(f"<{n_dims}i")
        name = data[off:off + ln].decode()
        off += ln
        cnt = int(np.prod(ne))
        dt = "<f4" if ftype == 0 else "<f2"
        arr = np.frombuffer(data, dt, cnt, off).reshape(tuple(reversed(ne)))
        off += cnt * (4 if ftype == 0 else 2)
        tensors[name] = arr
    return hp, filters, tensors


def f16(x):
    return np.asarray(x, np.float64).astype(np.float16).astype(np.float64)


def tables():
    x = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        gelu = f16(0.5 * x * (1.0 + np.tanh(0.7978845608028654 * x * (1.0 + 0.044715 * x * x))))
        expt = f16(np.exp(x))
    return gelu, expt


GELU, EXPT = tables()


def gelu(x):
    return GELU[np.asarray(x, np.float64).astype(np.float16).view(np.uint16)]


def table_exp(x):
    return EXPT[np.asarray(x, np.float64).astype(np.float16).view(np.uint16)]


def mel_spectrogram(pcm, filters, n_mel):
    n = pcm.size
    n_len = n // 160
    hann = 0.5 * (1.0 - np.cos(2.0 * np.pi * np.arange(400) / 400.0))
    out = np.zeros((n_mel, n_len))
    padded = np.concatenate([pcm.astype(np.float64), np.zeros(400)])
    for i in range(n_len):
        frame = hann * padded[i * 160:i * 160 + 400]
        spec = np.fft.fft(frame)
        p = spec.real ** 2 + spec.imag ** 2
        p[1:200] += p[399:200:-1]
        s = filters[:n_mel, :201] @ p[:201]
        out[:, i] = np.log10(np.maximum(s, 1e-10))
    mmax = out.max() - 8.0
    out = np.maximum(out, mmax)
    return ((out + 4.0) / 4.0).astype(np.float32)


def layer_norm(x, w, b):
    mean = x.mean(axis=-1, keepdims=True)
    var = ((x - mean) ** 2).mean(axis=-1, keepdims=True)
    return (x - mean) / np.sqrt(var + 1e-5) * w + b


def matmul(W, x):
    """ggml_mul_mat(W [out][in], x), exact products: an f16 W rounds x to f16;
    an f32 W (ftype-0 file, main.rs:817-821) takes x as it is."""
    xx = f16(x) if W.dtype == np.float16 else np.asarray(x, np.float64)
    return xx @ W.astype(np.float64).T


def attention(q, k, v, scale):
    """ggml softmax semantics: table exp of f16(s - max), normalise, f16 P."""
    s = (f16(q) @ f16(k).T) * scale
    p = table_exp(s - s.max(axis=-1, keepdims=True))
    p = f16(p / p.sum(axis=-1, keepdims=True))
    return p @ f16(v)


def encode(hp, T, mel):
    n, H = hp["n_audio_state"], hp["n_audio_head"]
    D = n // H
    X = np.zeros((hp["n_mels"], 2 * N_CTX))
    X[:, :min(2 * N_CTX, mel.shape[1])] = mel[:, :2 * N_CTX]
    # conv_1d_*_f16_f32 rounds its source to f16; the f32 kernel does not
    xp = np.pad(f16(X) if T["encoder.conv1.weight"].dtype == np.float16 else X, ((0, 0), (1, 1)))

    def conv(W, b, x, stride):
        Tout = (x.shape[1] - 2) // stride
        y = np.zeros((W.shape[0], Tout))
        Wf = W.astype(np.float64)
        for k in range(3):
            y += Wf[:, :, k] @ x[:, k:k + stride * Tout:stride]
        return gelu(y + b.reshape(-1, 1))

    g1 = conv(T["encoder.conv1.weight"], T["encoder.conv1.bias"], xp, 1)
    g2 = conv(T["encoder.conv2.weight"], T["encoder.conv2.bias"], np.pad(g1, ((0, 0), (1, 1))), 2)
    h = T["encoder.positional_embedding"][:N_CTX].astype(np.float64) + g2.T
    for i in range(hp["n_audio_layer"]):
        p = f"encoder.blocks.{i}."
        x = layer_norm(h, T[p + "attn_ln.weight"], T[p + "attn_ln.bias"])
        q = matmul(T[p + "attn.query.weight"], x) + T[p + "attn.query.bias"]
        k = matmul(T[p + "attn.key.weight"], x)
        v = matmul(T[p + "attn.value.weight"], x) + T[p + "attn.value.bias"]
        att = np.concatenate([attention(q[:, j * D:(j + 1) * D], k[:, j * D:(j + 1) * D], v[:, j * D:(j + 1) * D],
                                        1.0 / np.sqrt(D)) for j in range(H)], axis=1)
        h = h + matmul(T[p + "attn.out.weight"], att) + T[p + "attn.out.bias"]
        x = layer_norm(h, T[p + "mlp_ln.weight"], T[p + "mlp_ln.bias"])
        m = gelu(matmul(T[p + "mlp.0.weight"], x) + T[p + "mlp.0.bias"])
        h = h + matmul(T[p + "mlp.2.weight"], m) + T[p + "mlp.2.bias"]
    enc = layer_norm(h, T["encoder.ln_post.weight"], T["encoder.ln_post.bias"])
    sc = (n / H) ** -0.25
    ck, cv = [], []
    for l in range(hp["n_text_layer"]):
        p = f"decoder.blocks.{l}.cross_attn."
        ck.append((matmul(T[p + "key.weight"], enc) * sc).astype(np.float16))
        cv.append((matmul(T[p + "value.weight"], enc) + T[p + "value.bias"]).astype(np.float16))
    return enc.astype(np.float32), np.stack(ck), np.stack(cv)


def decode_logits(hp, T, ck, cv, tokens):
    n, H = hp["n_text_state"], hp["n_text_head"]
    D = n // H
    sc = (n / H) ** -0.25
    L = hp["n_text_layer"]
    kc = [np.zeros((0, n)) for _ in range(L)]
    vc = [np.zeros((0, n)) for _ in range(L)]
    te = T["decoder.token_embedding.weight"].astype(np.float64)
    out = []
    for pos, tok in enumerate(tokens):
        x = te[tok] + T["decoder.positional_embedding"][pos]
        for l in range(L):
            p = f"decoder.blocks.{l}."
            y = layer_norm(x, T[p + "attn_ln.weight"], T[p + "attn_ln.bias"])
            q = f16((matmul(T[p + "attn.query.weight"], y) + T[p + "attn.query.bias"]) * sc)
            kc[l] = np.vstack([kc[l], f16(matmul(T[p + "attn.key.weight"], y) * sc)])
            vc[l] = np.vstack([vc[l], f16(matmul(T[p + "attn.value.weight"], y) + T[p + "attn.value.bias"])])
            att = np.concatenate([attention(q[j * D:(j + 1) * D][None], kc[l][:, j * D:(j + 1) * D],
                                            vc[l][:, j * D:(j + 1) * D], 1.0)[0] for j in range(H)])
            x = x + matmul(T[p + "attn.out.weight"], att) + T[p + "attn.out.bias"]
            y = layer_norm(x, T[p + "cross_attn_ln.weight"], T[p + "cross_attn_ln.bias"])
            q = f16((matmul(T[p + "cross_attn.query.weight"], y) + T[p + "cross_attn.query.bias"]) * sc)
            K, V = ck[l].astype(np.float64), cv[l].astype(np.float64)
            att = np.concatenate([attention(q[j * D:(j + 1) * D][None], K[:, j * D:(j + 1) * D],
                                            V[:, j * D:(j + 1) * D], 1.0)[0] for j in range(H)])
            x = x + matmul(T[p + "cross_attn.out.weight"], att) + T[p + "cross_attn.out.bias"]
            y = layer_norm(x, T[p + "mlp_ln.weight"], T[p + "mlp_ln.bias"])
            m = gelu(matmul(T[p + "mlp.0.weight"], y) + T[p + "mlp.0.bias"])
            x = x + matmul(T[p + "mlp.2.weight"], m) + T[p + "mlp.2.bias"]
        y = layer_norm(x, T["decoder.ln.weight"], T["decoder.ln.bias"])
        out.append(matmul(te, y))
    return np.array(out)


def prompt(hp):
    sot, not_ = (50258, 50363) if hp["n_vocab"] >= 51865 else (50257, 50362)
    return [sot] + ([sot + 1, 50359] if hp["n_vocab"] >= 51865 else []) + [not_]


def greedy(hp, T, ck, cv, n_tok):
    eot = 50257 if hp["n_vocab"] >= 51865 else 50256
    toks = prompt(hp)
    np_ = len(toks)
    margins = []
    for _ in range(n_tok):
        lg = decode_logits(hp, T, ck, cv, toks)[-1]
        lg[eot] = -np.inf
        order = np.argsort(-lg, kind="stable")
        margins.append(lg[order[0]] - lg[order[1]])
        toks.append(int(order[0]))
    return np.array(toks[np_:], np.int32), np.array(margins)


def main(out_path=os.path.join(HERE, "micro_golden.npz"), quant=None):
    """quant "f32": the micro model as an ftype-0 (f32) file -> micro_f32_golden.npz"""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        mpath = os.path.join(d, "micro.bin")
        synth.write_ggml(mpath, "micro", quant=quant)
        sha = hashlib.sha256(open(mpath, "rb").read()).hexdigest()
        hp, filters, T = read_ggml(mpath)
    pcm = synth.synth_pcm_f32(SECONDS, SEED)
    mel = mel_spectrogram(pcm, filters, hp["n_mels"])
    enc, ck, cv = encode(hp, T, mel)
    toks, margins = greedy(hp, T, ck, cv, N_GREEDY)
    tf = np.array(prompt(hp) + list(range(1000, 1006)), np.int32)
    lg = decode_logits(hp, T, ck, cv, tf)
    top = np.argsort(-lg, axis=1, kind="stable")[:, :5]
    np.savez_compressed(out_path, model_sha256=np.array(sha), pcm_sha256=np.array(hashlib.sha256(pcm.tobytes()).hexdigest()),
                        n_ctx=N_CTX, mel=mel, enc=enc, ck=ck, cv=cv, greedy=toks, margins=margins,
                        tf_tokens=tf, tf_top5=top, tf_top5_logits=np.take_along_axis(lg, top, 1).astype(np.float32),
                        tf_logit_sum=lg.sum(1), tf_logit_abssum=np.abs(lg).sum(1))
    print(f"wrote {out_path}: greedy {toks.tolist()}")


if __name__ == "__main__":
    if "--f32" in sys.argv:
        main(os.path.join(HERE, "micro_f32_golden.npz"), quant="f32")
    else:
        main()
