"""Synthetic inputs for the Whisper hot path: ggml-v1 model files and 30 s clips.

Real ggml checkpoints and jfk.wav are not available offline, so
benchmarks and parity tests run on synthetic files with the real
hyper-parameters.  The file format is the one the reference loader reads:

  magic u32 0x67676d6c                                    /root/reference/src/main.rs:46, 368-371
  11 x i32 hparams                                        main.rs:623-633
  filters: i32 n_mel, i32 n_ff, f32[n_mel*n_ff]           main.rs:514-524
  vocab:   i32 n, n x (u32 len, bytes)                    main.rs:430, 579-583
  tensors: i32 n_dims, i32 name_len, i32 ftype, i32 ne[n_dims], name, data
                                                          main.rs:1385-1400, 1423-1437

Tensor set and storage dtypes follow WhisperModel::load (main.rs:947-1334):
matrices and conv kernels are f16 when hparams.f16 == 1; biases, LayerNorm
parameters, conv biases ([1, n]) and both positional embeddings are f32.

Value recipe: 2-D+ weights N(0, 0.02) f16, biases N(0, 0.01),
LN gains 1 + N(0, 0.02), encoder PE sinusoidal, decoder PE N(0, 0.01),
Slaney filterbank, seed = crc32(tensor name).  Audio: SURVEY.md §8d formula,
quantised to int16 and read back as s16/32768 (main.rs:1673-1679).
"""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

GGML_MAGIC = 0x67676D6C
SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160

# name -> (n_vocab, n_audio_ctx, n_state, n_head, n_layer, n_text_ctx, n_mels)
MODEL_DIMS = {
    "micro":    dict(n_vocab=51864, n_audio_ctx=1500, n_audio_state=128,  n_audio_head=2,  n_audio_layer=2,
                     n_text_ctx=448, n_text_state=128,  n_text_head=2,  n_text_layer=2,  n_mels=80),
    "tiny.en":  dict(n_vocab=51864, n_audio_ctx=1500, n_audio_state=384,  n_audio_head=6,  n_audio_layer=4,
                     n_text_ctx=448, n_text_state=384,  n_text_head=6,  n_text_layer=4,  n_mels=80),
    "tiny":     dict(n_vocab=51865, n_audio_ctx=1500, n_audio_state=384,  n_audio_head=6,  n_audio_layer=4,
                     n_text_ctx=448, n_text_state=384,  n_text_head=6,  n_text_layer=4,  n_mels=80),
    "base":     dict(n_vocab=51865, n_audio_ctx=1500, n_audio_state=512,  n_audio_head=8,  n_audio_layer=6,
                     n_text_ctx=448, n_text_state=512,  n_text_head=8,  n_text_layer=6,  n_mels=80),
    "small":    dict(n_vocab=51865, n_audio_ctx=1500, n_audio_state=768,  n_audio_head=12, n_audio_layer=12,
                     n_text_ctx=448, n_text_state=768,  n_text_head=12, n_text_layer=12, n_mels=80),
    "medium":   dict(n_vocab=51865, n_audio_ctx=1500, n_audio_state=1024, n_audio_head=16, n_audio_layer=24,
                     n_text_ctx=448, n_text_state=1024, n_text_head=16, n_text_layer=24, n_mels=80),
    "large-v3": dict(n_vocab=51866, n_audio_ctx=1500, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                     n_text_ctx=448, n_text_state=1280, n_text_head=20, n_text_layer=32, n_mels=128),
}

HPARAM_ORDER = ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer", "n_mels", "f16")


# ----------------------------------------------------------------------------
# Slaney mel filterbank (librosa.filters.mel(htk=False, norm="slaney") algorithm)
# ----------------------------------------------------------------------------
def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(n_mels: int, n_fft: int = N_FFT, sr: int = SAMPLE_RATE) -> np.ndarray:
    """[n_mels][1 + n_fft/2] float32, row-major as WhisperFilters::load reads it (main.rs:513-535)."""
    n_freq = 1 + n_fft // 2
    fftfreqs = np.linspace(0, sr / 2, n_freq)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, n_freq), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w.astype(np.float32)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Whisper encoder positional embedding, [length][channels] float32."""
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2))
    t = np.arange(length)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


# ----------------------------------------------------------------------------
# tensor list (same names/shapes as WhisperModel::load, main.rs:947-1334)
# ----------------------------------------------------------------------------
def tensor_specs(hp: dict):
    """Yield (name, torch_shape, kind) with kind in {w, b, g, lnb, epe, dpe}.

    torch_shape is row-major (outermost first); the file stores ne reversed.
    """
    n = hp["n_audio_state"]
    nt = hp["n_text_state"]
    yield "encoder.positional_embedding", (hp["n_audio_ctx"], n), "epe"
    yield "encoder.conv1.weight", (n, hp["n_mels"], 3), "w"
    yield "encoder.conv1.bias", (n, 1), "b"
    yield "encoder.conv2.weight", (n, n, 3), "w"
    yield "encoder.conv2.bias", (n, 1), "b"
    for i in range(hp["n_audio_layer"]):
        p = f"encoder.blocks.{i}."
        yield p + "attn_ln.weight", (n,), "g"
        yield p + "attn_ln.bias", (n,), "lnb"
        yield p + "attn.query.weight", (n, n), "w"
        yield p + "attn.query.bias", (n,), "b"
        yield p + "attn.key.weight", (n, n), "w"
        yield p + "attn.value.weight", (n, n), "w"
        yield p + "attn.value.bias", (n,), "b"
        yield p + "attn.out.weight", (n, n), "w"
        yield p + "attn.out.bias", (n,), "b"
        yield p + "mlp_ln.weight", (n,), "g"
        yield p + "mlp_ln.bias", (n,), "lnb"
        yield p + "mlp.0.weight", (4 * n, n), "w"
        yield p + "mlp.0.bias", (4 * n,), "b"
        yield p + "mlp.2.weight", (n, 4 * n), "w"
        yield p + "mlp.2.bias", (n,), "b"
    yield "encoder.ln_post.weight", (n,), "g"
    yield "encoder.ln_post.bias", (n,), "lnb"
    yield "decoder.positional_embedding", (hp["n_text_ctx"], nt), "dpe"
    yield "decoder.token_embedding.weight", (hp["n_vocab"], nt), "w"
    for i in range(hp["n_text_layer"]):
        p = f"decoder.blocks.{i}."
        for a in ("attn", "cross_attn"):
            yield p + f"{a}_ln.weight", (nt,), "g"
            yield p + f"{a}_ln.bias", (nt,), "lnb"
            yield p + f"{a}.query.weight", (nt, nt), "w"
            yield p + f"{a}.query.bias", (nt,), "b"
            yield p + f"{a}.key.weight", (nt, nt), "w"
            yield p + f"{a}.value.weight", (nt, nt), "w"
            yield p + f"{a}.value.bias", (nt,), "b"
            yield p + f"{a}.out.weight", (nt, nt), "w"
            yield p + f"{a}.out.bias", (nt,), "b"
        yield p + "mlp_ln.weight", (nt,), "g"
        yield p + "mlp_ln.bias", (nt,), "lnb"
        yield p + "mlp.0.weight", (4 * nt, nt), "w"
        yield p + "mlp.0.bias", (4 * nt,), "b"
        yield p + "mlp.2.weight", (nt, 4 * nt), "w"
        yield p + "mlp.2.bias", (nt,), "b"
    yield "decoder.ln.weight", (nt,), "g"
    yield "decoder.ln.bias", (nt,), "lnb"


def tensor_value(name: str, shape, kind: str, hp: dict, wscale: float = 0.02, wf32: bool = False) -> np.ndarray:
    """wf32: weight matrices / conv kernels stay f32 (an ftype-0 file; values
    not representable in f16, so a path that rounded them would show)."""
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    if kind == "w":
        w = rng.standard_normal(shape, dtype=np.float32) * wscale
        return w.astype(np.float32) if wf32 else w.astype(np.float16)
    if kind in ("b", "lnb"):
        return (rng.standard_normal(shape, dtype=np.float32) * 0.01).astype(np.float32)
    if kind == "g":
        return (1.0 + rng.standard_normal(shape, dtype=np.float32) * 0.02).astype(np.float32)
    if kind == "epe":
        return sinusoids(shape[0], shape[1])
    if kind == "dpe":
        return (rng.standard_normal(shape, dtype=np.float32) * 0.01).astype(np.float32)
    raise ValueError(kind)


def _vocab_tokens(n: int):
    for i in range(n):
        yield (f" w{i}" if i < 50256 else f"<|special{i}|>").encode()


# ----------------------------------------------------------------------------
# ggml quantisation (QNT version 2 block layouts)
# ----------------------------------------------------------------------------
GGML_QNT_VERSION = 2
QUANT_TYPES = {"q4_0": (2, 2), "q4_1": (3, 3), "q5_0": (6, 8), "q5_1": (7, 9), "q8_0": (8, 7)}  # -> (ttype, ftype)


def _absmax_signed(x):
    """ggml's 'max by absolute value, keeping the sign' per row of 32."""
    i = np.abs(x).argmax(axis=1)
    return x[np.arange(x.shape[0]), i]


def _inv(d):
    with np.errstate(divide="ignore"):
        return np.where(d != 0, np.float32(1.0) / np.where(d != 0, d, np.float32(1.0)), np.float32(0.0)).astype(np.float32)


def _qh_bits(q):
    bits = np.arange(32, dtype=np.uint64)
    return ((((q & 0x10) >> 4).astype(np.uint64) << bits).sum(axis=1)).astype("<u4")


def quantize(w: np.ndarray, qtype: str) -> bytes:
    """ggml quantize_row_<type>_ref (QNT v2 layouts) over rows of 32 weights."""
    if qtype == "q5_1":
        return quantize_q5_1(w)
    x = np.ascontiguousarray(w, dtype=np.float32).reshape(-1, 32)
    nb = x.shape[0]
    if qtype == "q8_0":
        d = np.abs(x).max(axis=1) / np.float32(127.0)
        q = np.round(x * _inv(d)[:, None])  # roundf: half away from zero
        q = np.where(np.abs(x * _inv(d)[:, None] - np.trunc(x * _inv(d)[:, None])) == 0.5,
                     np.trunc(x * _inv(d)[:, None]) + np.sign(x), q)
        blk = np.zeros(nb, dtype=[("d", "<f2"), ("qs", "i1", 32)])
        blk["d"] = d.astype(np.float16)
        blk["qs"] = q.astype(np.int8)
        return blk.tobytes()
    if qtype in ("q4_0", "q5_0"):
        lv = 8 if qtype == "q4_0" else 16
        d = _absmax_signed(x) / np.float32(-lv)
        q = np.minimum(2 * lv - 1, (x * _inv(d)[:, None] + np.float32(lv + 0.5)).astype(np.int8).astype(np.int64))
    else:  # q4_1
        mn = x.min(axis=1)
        d = (x.max(axis=1) - mn) / np.float32(15.0)
        q = np.minimum(15, ((x - mn[:, None]) * _inv(d)[:, None] + np.float32(0.5)).astype(np.int8).astype(np.int64))
    q &= 0xFF
    qs = ((q[:, :16] & 0x0F) | ((q[:, 16:] & 0x0F) << 4)).astype(np.uint8)
    if qtype == "q4_0":
        blk = np.zeros(nb, dtype=[("d", "<f2"), ("qs", "u1", 16)])
    elif qtype == "q4_1":
        blk = np.zeros(nb, dtype=[("d", "<f2"), ("m", "<f2"), ("qs", "u1", 16)])
        blk["m"] = mn.astype(np.float16)
    else:
        blk = np.zeros(nb, dtype=[("d", "<f2"), ("qh", "<u4"), ("qs", "u1", 16)])
        blk["qh"] = _qh_bits(np.concatenate([q[:, :16], q[:, 16:]], axis=1))
    blk["d"] = d.astype(np.float16)
    blk["qs"] = qs
    return blk.tobytes()


def quantize_q5_1(w: np.ndarray) -> bytes:
    """ggml quantize_row_q5_1_ref over rows of 32: {f16 d, f16 m, u32 qh, u8 qs[16]}.
    f32 arithmetic as in ggml: d = (max - min) / 31, q = (int)((x - min) * (1/d) + 0.5);
    element j < 16 in the low nibble of qs[j], element j + 16 in its high nibble,
    bit 4 of element j in bit j of qh."""
    x = np.ascontiguousarray(w, dtype=np.float32).reshape(-1, 32)
    mn = x.min(axis=1)
    mx = x.max(axis=1)
    d = (mx - mn) / np.float32(31.0)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / np.where(d != 0, d, np.float32(1.0)), np.float32(0.0)).astype(np.float32)
    q = (((x - mn[:, None]) * idv[:, None]) + np.float32(0.5)).astype(np.int64) & 0xFF  # (uint8_t) cast
    lo, hi = q[:, :16], q[:, 16:]
    qs = ((lo & 0x0F) | ((hi & 0x0F) << 4)).astype(np.uint8)
    bits = np.arange(16, dtype=np.uint64)
    qh = ((((lo & 0x10) >> 4).astype(np.uint64) << bits).sum(axis=1) +
          (((hi & 0x10) >> 4).astype(np.uint64) << (bits + 16)).sum(axis=1)).astype("<u4")
    blk = np.zeros(x.shape[0], dtype=[("d", "<f2"), ("m", "<f2"), ("qh", "<u4"), ("qs", "u1", 16)])
    blk["d"] = d.astype(np.float16)
    blk["m"] = mn.astype(np.float16)
    blk["qh"] = qh
    blk["qs"] = qs
    return blk.tobytes()


def write_ggml(path: str, model: str = "base", hp_override: dict | None = None,
               wscale: float = 0.02, n_vocab_file: int | None = None, tensor_hook=None,
               quant: str | None = None) -> dict:
    """Write a synthetic ggml-v1 Whisper file; returns the hparams used.
    tensor_hook(name, array) -> array may edit tensors before they are written.
    quant "f32" writes an ftype-0 file (hparams.f16 = 0: every matrix and conv
    kernel f32, main.rs:817-821); "q5_1", "q8_0", ... store every 2-D weight matrix in that ggml block format,
    as whisper.cpp's quantize tool does (conv kernels, biases, LN parameters
    and positional embeddings keep their type); hparams.f16 then carries the
    file ftype + 1000 * GGML_QNT_VERSION."""
    hp = dict(MODEL_DIMS[model])
    wf32 = quant == "f32"
    if wf32:
        quant = None
    hp["f16"] = (0 if wf32 else 1) if quant is None else QUANT_TYPES[quant][1] + 1000 * GGML_QNT_VERSION
    if hp_override:
        hp.update(hp_override)
    n_vocab_file = 50257 if n_vocab_file is None else n_vocab_file
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<I", GGML_MAGIC))
        f.write(struct.pack("<11i", *[hp[k] for k in HPARAM_ORDER]))
        filt = mel_filterbank(hp["n_mels"])
        f.write(struct.pack("<ii", filt.shape[0], filt.shape[1]))
        f.write(filt.astype("<f4").tobytes())
        f.write(struct.pack("<i", n_vocab_file))
        for tok in _vocab_tokens(n_vocab_file):
            f.write(struct.pack("<I", len(tok)))
            f.write(tok)
        for name, shape, kind in tensor_specs(hp):
            arr = tensor_value(name, shape, kind, hp, wscale, wf32=wf32)
            if tensor_hook is not None:
                arr = tensor_hook(name, arr)
            ftype = 1 if arr.dtype == np.float16 else 0
            ne = tuple(reversed(shape))
            nb = name.encode()
            if quant is not None and kind == "w" and len(shape) == 2:
                ftype = QUANT_TYPES[quant][0]
                payload = quantize(arr.astype(np.float32), quant)
            else:
                payload = arr.astype("<f2" if ftype else "<f4").tobytes()
            f.write(struct.pack("<iii", len(ne), len(nb), ftype))
            f.write(struct.pack(f"<{len(ne)}i", *ne))
            f.write(nb)
            f.write(payload)
    os.replace(tmp, path)
    return hp


SHARP_TE, SHARP_PE = 4.0, 100.0


def sharp_hook(name: str, arr: np.ndarray) -> np.ndarray:
    """The "-sharp" variants (e.g. "base-sharp"): decoder.token_embedding x 4
    and decoder.positional_embedding x 100 (sigma 0.08 and 1.0).  The random
    models' logits then spread widely and depend on the position, so greedy
    decoding emits a long, varied id sequence whose top-2 margins stay far
    above f32 reordering noise (base: ~95 distinct ids in 96 steps, smallest
    margin ~8e-3; large-v3 5-beam: every selection margin >= 1e-2 over 40
    steps) — a long decode horizon the parity tests can compare id for id."""
    if name == "decoder.token_embedding.weight":
        return (arr.astype(np.float32) * SHARP_TE).astype(arr.dtype)
    if name == "decoder.positional_embedding":
        return (arr.astype(np.float32) * SHARP_PE).astype(arr.dtype)
    return arr


XSHARP_CONV1, XSHARP_PE = 20.0, 3.0


def xsharp_hook(name: str, arr: np.ndarray) -> np.ndarray:
    """The "-xsharp" variants (e.g. "base-xsharp"): a model whose greedy ids
    follow the audio.  In the plain random model the encoder input is
    dominated by its sinusoidal positional embedding (conv1 maps the
    normalised mel to ~0.3 per channel, the embedding is ~0.7), so every
    clip's encoder output, cross K / V and ids are nearly the same (base,
    SURVEY clips 1234..1241: 1-2 distinct id sequences).  Here conv1's
    kernel is x 20, so the mel dominates the encoder, and the decoder's
    positional embedding x 3 (sigma 0.03) varies the ids along the sequence.
    With tone clips (synth_pcm_tones) the oracle gives 8 distinct 64-token
    greedy sequences over seeds 1234..1241 at the plain model's logit noise
    floor (|ggml order - exact dots| 1.2e-3).  The cross-attention sharpening
    first tried (query / key x 8, out x 10) made the ids audio-dependent too
    but chaotic: device and oracle logits 0.2-0.34 apart, free-running ids
    parting after 2-84 tokens (profiles/r05/xsharp_qk8_probe.log)."""
    if name == "encoder.conv1.weight":
        return (arr.astype(np.float32) * XSHARP_CONV1).astype(arr.dtype)
    if name == "decoder.positional_embedding":
        return (arr.astype(np.float32) * XSHARP_PE).astype(arr.dtype)
    return arr


XSHARP_LV3_PE, XSHARP_LV3_LNW, XSHARP_LV3_CO = 5.0, 16.0, 3.0


def xsharp_lv3_hook(name: str, arr: np.ndarray) -> np.ndarray:
    """"large-v3-xsharp": conv1 x 20 (as xsharp_hook: the mel dominates the
    encoder), the decoder positional embedding x 5, every decoder layer's
    cross-attention output projection x 3 (the audio dominates the decoder's
    residual: each clip settles on its own id) and the decoder's final
    LayerNorm weight x 16 (every logit spreads 16x; scaling the tied token
    embedding instead makes the input token dominate the residual and the
    model repeat its first id).  The oracle (scripts/xsharp_probe.py,
    profiles/r06/xsharp_lv3_probe.log): 6 distinct 24-token greedy sequences
    over tone clips 1234-1241 (xsharp_hook alone: the 5-beam selections meet
    a margin below 2e-3 within 3-5 steps and 4 of the 8 clips share ids), and
    a 5-beam search on clip 1234 whose 40 selection margins all exceed 2e-3."""
    if name == "decoder.ln.weight":
        return (arr.astype(np.float32) * XSHARP_LV3_LNW).astype(arr.dtype)
    if name == "decoder.positional_embedding":
        return (arr.astype(np.float32) * XSHARP_LV3_PE).astype(arr.dtype)
    if name.startswith("decoder.blocks.") and name.endswith(".cross_attn.out.weight"):
        return (arr.astype(np.float32) * XSHARP_LV3_CO).astype(arr.dtype)
    if name == "encoder.conv1.weight":
        return (arr.astype(np.float32) * XSHARP_CONV1).astype(arr.dtype)
    return arr


LNMEAN_OFFSET = 16.0


def lnmean_hook(name: str, arr: np.ndarray) -> np.ndarray:
    """The "-lnmean" variants: decoder.positional_embedding + 16, so every
    decoder residual row (token + position embedding, then the layers' sums)
    has a mean of ~16 over a spread of ~0.02-0.1: |mean| / std up to ~700
    at the first LayerNorm.  LayerNorm removes the offset, so the model is
    the plain one up to rounding; it exercises the persistent decoder's
    one-pass statistics (E[x^2] - mean^2 in double) against the oracle's
    two-pass ggml norm where cancellation is largest (tests/test_ln_formula.py
    states the bound, mean^2 / var <= 1e6)."""
    if name == "decoder.positional_embedding":
        return (arr.astype(np.float32) + np.float32(LNMEAN_OFFSET)).astype(arr.dtype)
    return arr


def tensor_table(path: str) -> dict:
    """{name: (byte offset of the data, dtype, torch shape)} of an f16 / f32
    ggml file written by write_ggml (no quantised tensors)."""
    out = {}
    with open(path, "rb") as f:
        f.seek(4 + 11 * 4)
        n_mel, n_fft = struct.unpack("<ii", f.read(8))
        f.seek(n_mel * n_fft * 4, 1)
        (n_tok,) = struct.unpack("<i", f.read(4))
        for _ in range(n_tok):
            (ln,) = struct.unpack("<I", f.read(4))
            f.seek(ln, 1)
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                break
            nd, nl, ft = struct.unpack("<iii", hdr)
            if ft not in (0, 1):
                raise ValueError(f"{path}: tensor type {ft} is not f32 / f16")
            ne = struct.unpack(f"<{nd}i", f.read(4 * nd))
            name = f.read(nl).decode()
            dt = np.dtype("<f2" if ft else "<f4")
            shape = tuple(reversed(ne))
            out[name] = (f.tell(), dt, shape)
            f.seek(int(np.prod(shape)) * dt.itemsize, 1)
    return out


def derive_variant(src: str, dst: str, tensor_hook) -> None:
    """The file write_ggml(dst, <src's model>, tensor_hook=tensor_hook) would
    write, made from src (the same model written without a hook): a copy
    with the tensors the hook changes rewritten in place.  write_ggml stores
    every generated array in its own dtype, so reading it back gives the
    array the hook would have seen (bitwise; tests/test_quant.py checks the
    two routes agree), and the hooks keep the dtype, so sizes and offsets do
    not move.  A large-v3 variant takes seconds instead of regenerating 1.5 G
    random weights (~50 s of a GPU session's time)."""
    import shutil
    tmp = f"{dst}.tmp{os.getpid()}"
    shutil.copyfile(src, tmp)
    with open(tmp, "r+b") as f:
        for name, (off, dt, shape) in tensor_table(src).items():
            f.seek(off)
            arr = np.frombuffer(f.read(int(np.prod(shape)) * dt.itemsize), dt).reshape(shape)
            new = tensor_hook(name, arr.astype(dt.newbyteorder("=")))
            if new is arr or np.array_equal(new.view(np.uint8), arr.view(np.uint8)):
                continue
            assert new.dtype == arr.dtype and new.shape == arr.shape, name
            f.seek(off)
            f.write(np.ascontiguousarray(new).astype(dt).tobytes())
    os.replace(tmp, dst)


def model_path(model: str, cache_dir: str | None = None) -> str:
    """Generate (once) and return the path of a synthetic model file."""
    cache_dir = cache_dir or os.environ.get("WMI_MODEL_CACHE", "/tmp/wmi_models")
    os.makedirs(cache_dir, exist_ok=True)
    p = os.path.join(cache_dir, f"ggml-synth-{model}.bin")
    if not os.path.exists(p):
        base, _, quant = model.partition("-q")
        if model.endswith("-lnmean"):
            derive_variant(model_path(model[:-7], cache_dir), p, lnmean_hook)
        elif model.endswith("-xsharp"):
            derive_variant(model_path(model[:-7], cache_dir), p,
                           xsharp_lv3_hook if model == "large-v3-xsharp" else xsharp_hook)
        elif model.endswith("-sharp"):
            derive_variant(model_path(model[:-6], cache_dir), p, sharp_hook)
        elif model.endswith("-f32"):  # e.g. "micro-f32": an ftype-0 (f32) file
            write_ggml(p, model[:-4], quant="f32")
        elif quant:  # e.g. "small-q5_1": the small model's weights in ggml q5_1
            write_ggml(p, base, quant="q" + quant)
        else:
            write_ggml(p, model)
    return p


# ----------------------------------------------------------------------------
# synthetic audio
# ----------------------------------------------------------------------------
def synth_pcm_i16(seconds: float = 30.0, seed: int = 1234) -> np.ndarray:
    n = int(round(seconds * SAMPLE_RATE))
    t = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(seed)
    x = (0.4 * np.sin(2 * np.pi * 220 * t / SAMPLE_RATE) * (0.6 + 0.4 * np.sin(2 * np.pi * 0.5 * t / SAMPLE_RATE))
         + 0.2 * np.sin(2 * np.pi * 1330 * t / SAMPLE_RATE) + 0.05 * rng.standard_normal(n))
    x = np.clip(x, -1.0, 1.0)
    return np.round(x * 32767).astype(np.int16)


def pcm_i16_to_f32(s16: np.ndarray) -> np.ndarray:
    """convert_integer_to_float_audio (main.rs:1673-1679): s / 32768.0 in f32."""
    return (s16.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def synth_pcm_f32(seconds: float = 30.0, seed: int = 1234) -> np.ndarray:
    return pcm_i16_to_f32(synth_pcm_i16(seconds, seed))


def synth_pcm_tones(seconds: float = 30.0, seed: int = 1234) -> np.ndarray:
    """Clips whose content differs with the seed (the SURVEY §8d clips share
    their tones and differ only in the noise): two tones at seed-drawn
    frequencies (150-600 Hz, amplitude-modulated at 0.2-2 Hz, and 0.8-3 kHz)
    plus the same 0.05 N(0, 1) noise; int16-quantised, then s / 32768."""
    n = int(round(seconds * SAMPLE_RATE))
    t = np.arange(n, dtype=np.float64) / SAMPLE_RATE
    rng = np.random.default_rng(seed)
    f1, f2 = rng.uniform(150, 600), rng.uniform(800, 3000)
    am = 0.5 + 0.5 * np.sin(2 * np.pi * rng.uniform(0.2, 2) * t)
    x = 0.4 * np.sin(2 * np.pi * f1 * t) * am + 0.2 * np.sin(2 * np.pi * f2 * t) + 0.05 * rng.standard_normal(n)
    return pcm_i16_to_f32(np.round(np.clip(x, -1.0, 1.0) * 32767).astype(np.int16))


def write_wav(path: str, s16: np.ndarray, sr: int = SAMPLE_RATE) -> None:
    """16-bit mono PCM WAV (what hound reads in main.rs:2067-2068)."""
    data = s16.astype("<i2").tobytes()
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sr, sr * 2, 2, 16))
        f.write(b"data" + struct.pack("<I", len(data)) + data)
