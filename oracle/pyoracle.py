"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
(as the checker / CPU baseline).  The product path never imports this file.
PARITY UNPINNED: see oracle/README.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WMI_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # (sanitizer builds)
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i32, sz = C.c_void_p, C.c_int32, C.c_size_t
        fp = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        hp_ = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.or_load.argtypes = [C.c_char_p, C.POINTER(vp), C.c_char_p, sz]
        L.or_free.argtypes = [vp]
        L.or_get_hparams.argtypes = [vp, ip]
        L.or_special_tokens.argtypes = [vp, ip]
        L.or_prompt.argtypes = [vp, ip]
        L.or_tables.argtypes = [hp_, hp_]
        L.or_set_dot_mode.argtypes = [C.c_int]
        L.or_mel.argtypes = [vp, fp, sz, C.c_int, C.c_void_p, C.POINTER(i32)]
        L.or_checksums.argtypes = [vp, fp, sz, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.or_encode.argtypes = [vp, fp, i32, C.c_int, C.c_int, C.c_int, fp, hp_, hp_, C.c_void_p]
        L.or_decode_logits.argtypes = [vp, hp_, hp_, C.c_int, ip, C.c_int, C.c_int, fp]
        L.or_decode_greedy.argtypes = [vp, hp_, hp_, C.c_int, C.c_int, C.c_int, C.c_int, ip, C.POINTER(i32), fp]
        L.or_dequant.argtypes = [C.c_int, C.c_void_p, C.c_int64, hp_]
        L.or_decode_beam.argtypes = [vp, hp_, hp_, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, ip, C.POINTER(i32),
                                     C.POINTER(C.c_double), C.POINTER(C.c_float), fp, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


HP_NAMES = ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
            "n_text_state", "n_text_head", "n_text_layer", "n_mels", "f16")


class OracleError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def set_dot_mode(exact_double: bool) -> None:
    """Switch dot-product accumulation (noise-floor measurement only)."""
    lib().or_set_dot_mode(int(exact_double))


def dequant(qtype: int, blocks: bytes, nel: int) -> np.ndarray:
    """The oracle loader's dequantisation (f16 bits) of ggml blocks."""
    out = np.zeros(nel, np.uint16)
    buf = C.create_string_buffer(bytes(blocks), len(blocks))
    rc = lib().or_dequant(qtype, C.cast(buf, C.c_void_p), nel, out)
    if rc:
        raise OracleError(rc, "dequant")
    return out


def tables():
    g = np.zeros(65536, np.uint16)
    e = np.zeros(65536, np.uint16)
    lib().or_tables(g, e)
    return g, e


class OracleModel:
    def __init__(self, path: str):
        self.h = None
        self.path = path
        L = lib()
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = L.or_load(path.encode(), C.byref(h), err, 512)
        if rc != 0:
            raise OracleError(rc, err.value.decode())
        self.h = h
        hp = np.zeros(11, np.int32)
        L.or_get_hparams(h, hp)
        self.hp = dict(zip(HP_NAMES, (int(x) for x in hp)))
        sp = np.zeros(9, np.int32)
        L.or_special_tokens(h, sp)
        self.special = dict(zip(("eot", "sot", "prev", "solm", "not", "beg", "translate", "transcribe",
                                 "multilingual"), (int(x) for x in sp)))

    def close(self):
        if self.h:
            lib().or_free(self.h)
            self.h = None

    __del__ = close

    def prompt(self):
        out = np.zeros(8, np.int32)
        n = lib().or_prompt(self.h, out)
        return out[:n].tolist()

    def mel(self, pcm: np.ndarray, n_threads: int = 4) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.float32)
        n_len = C.c_int32()
        lib().or_mel(self.h, pcm, pcm.size, n_threads, None, C.byref(n_len))
        out = np.zeros((self.hp["n_mels"], n_len.value), np.float32)
        rc = lib().or_mel(self.h, pcm, pcm.size, n_threads, out.ctypes.data, C.byref(n_len))
        if rc:
            raise OracleError(rc, "mel")
        return out

    def checksums(self, pcm: np.ndarray, mel_offset: int = 0, n_ctx: int = 0, n_threads: int = 4) -> dict:
        """The reference's debug sums (main.rs:1571, 1686, 1690, 1647, 1832)."""
        pcm = np.ascontiguousarray(pcm, np.float32)
        out = np.zeros(5, np.float32)
        rc = lib().or_checksums(self.h, pcm, pcm.size, mel_offset, n_ctx or self.hp["n_audio_ctx"], n_threads,
                                out.ctypes.data)
        if rc:
            raise OracleError(rc, "checksums")
        return dict(zip(("hann", "samples", "filters", "mel_raw", "mel_window"), out.tolist()))

    def encode(self, mel: np.ndarray, n_ctx: int = 0, mel_offset: int = 0, n_threads: int = 8, probe: bool = False):
        hp = self.hp
        n_ctx = n_ctx or hp["n_audio_ctx"]
        n = hp["n_audio_state"]
        mel = np.ascontiguousarray(mel, np.float32)
        enc = np.zeros((n_ctx, n), np.float32)
        ck = np.zeros((hp["n_text_layer"], n_ctx, hp["n_text_state"]), np.uint16)
        cv = np.zeros_like(ck)
        pr = np.zeros((hp["n_audio_layer"] + 1, n_ctx, n), np.float32) if probe else None
        rc = lib().or_encode(self.h, mel, mel.shape[1], mel_offset, n_ctx, n_threads, enc, ck, cv,
                             pr.ctypes.data if probe else None)
        if rc:
            raise OracleError(rc, "encode")
        return (enc, ck, cv, pr) if probe else (enc, ck, cv)

    def decode_logits(self, ck, cv, tokens, n_threads: int = 8) -> np.ndarray:
        tokens = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros((tokens.size, self.hp["n_vocab"]), np.float32)
        rc = lib().or_decode_logits(self.h, ck, cv, ck.shape[1], tokens, tokens.size, n_threads, out)
        if rc:
            raise OracleError(rc, "decode_logits")
        return out

    def decode_greedy(self, ck, cv, max_tokens: int, suppress_eot: bool = False, n_threads: int = 8):
        toks = np.zeros(max_tokens, np.int32)
        margins = np.zeros(max_tokens, np.float32)
        n = C.c_int32()
        rc = lib().or_decode_greedy(self.h, ck, cv, ck.shape[1], max_tokens, int(suppress_eot), n_threads, toks,
                                    C.byref(n), margins)
        if rc:
            raise OracleError(rc, "decode_greedy")
        return toks[:n.value], margins[:n.value]

    def decode_beam(self, ck, cv, beam: int, max_tokens: int, suppress_eot: bool = False, n_threads: int = 8,
                    step_gaps: bool = False, trace: bool = False):
        """Beam search (wmi_oracle.h): (tokens, score, smallest selection margin),
        plus each step's selection margin when step_gaps, plus with trace a
        dict: "logits" [steps][beam][V] (each active hypothesis' logits before
        EOT suppression, NaN rows where inactive), "sel" [steps][beam][2]
        ((parent, token) of the slots after each step, -1 where unfilled)."""
        toks = np.zeros(max_tokens + 1, np.int32)
        n = C.c_int32()
        score = C.c_double()
        gap = C.c_float()
        sg = np.zeros(max_tokens, np.float32)
        tr = None
        if trace:
            tr = {"logits": np.full((max_tokens, beam, self.hp["n_vocab"]), np.nan, np.float32),
                  "sel": np.full((max_tokens, beam, 2), -1, np.int32)}
        rc = lib().or_decode_beam(self.h, ck, cv, ck.shape[1], beam, max_tokens, int(suppress_eot), n_threads, toks,
                                  C.byref(n), C.byref(score), C.byref(gap), sg,
                                  tr["logits"].ctypes.data if trace else None, tr["sel"].ctypes.data if trace else None)
        if rc:
            raise OracleError(rc, "decode_beam")
        out = (toks[:n.value], score.value, gap.value) + ((sg,) if step_gaps else ())
        return out + (tr,) if trace else out


# ---------------------------------------------------------------------------
# Timestamp decoding and whisper_full windows.  Neither
# exists in the reference (it declares WhisperTokenData / WhisperSegment,
# main.rs:317-331, 599-604, and exp_n_audio_ctx / mel_offset windowing,
# main.rs:362, 1822-1823, but no loop); the semantics restated here are
# whisper.cpp-1.0.3's whisper_sample_timestamp / whisper_sample_best /
# whisper_full, which the reference's structs follow.  Parity unpinned beyond
# this restatement.  float64 softmax over the f32 logits.
# ---------------------------------------------------------------------------
def ts_sample(logits, special, first: bool):
    """One sampled token: (record dict, decision margin).  margin = the
    smaller of the top-2 logit gap in the chosen candidate set and the
    relative gap of the timestamp-vs-text test (0 for the forced first one)."""
    l32 = np.asarray(logits, np.float32)
    l = l32.astype(np.float64)
    mx = float(l32.max())
    e = np.exp(l - mx)
    Z = e.sum()
    beg = special["beg"]
    ts = e[beg:].sum() / Z
    id_ts = beg + int(np.argmax(l32[beg:]))
    id_tx = int(np.argmax(l32[:beg]))
    p_tx = e[id_tx] / Z
    if first:
        cand = np.arange(beg + 1, l.size)
        dec_margin = np.inf
    elif ts > p_tx:
        cand = np.arange(beg, l.size)
        dec_margin = abs(ts - p_tx) / max(ts, p_tx)
    else:
        mask = np.ones(l.size, bool)
        mask[[special["sot"], special["solm"], special["not"]]] = False
        cand = np.nonzero(mask)[0]
        dec_margin = abs(ts - p_tx) / max(ts, p_tx)
    vals = l32[cand]
    k = int(np.argmax(vals))
    tid = int(cand[k])
    srt = np.sort(vals)
    gap = float(srt[-1] - srt[-2]) if srt.size > 1 else np.inf
    rec = {"id": tid, "tid": id_ts, "p": e[tid] / Z, "pt": (e[id_ts] / Z) / (ts + 1e-10), "ptsum": ts}
    return rec, min(gap, dec_margin)


def ts_window_ref(om, ck, cv, prompt, max_tokens, n_threads=8):
    """One window (wmi_decode_timestamps): records and the smallest margin.
    Teacher-forced logits of prompt + tokens so far at every step."""
    toks, recs, margin = list(prompt), [], np.inf
    for t in range(max_tokens):
        lg = om.decode_logits(ck, cv, np.array(toks, np.int32), n_threads=n_threads)[-1]
        r, m = ts_sample(lg, om.special, t == 0)
        recs.append(r)
        margin = min(margin, m)
        toks.append(r["id"])
        if r["id"] == om.special["eot"]:
            break
    return recs, margin


def transcribe_ref(om, pcm, n_ctx, max_tokens, token_text, n_threads=8):
    """whisper_full restated (wmi_api.cpp run_transcribe): segments
    [{t0, t1, text, ids}] and the smallest sampling margin met."""
    sp, hp = om.special, om.hp
    mel = om.mel(pcm, n_threads=4)
    n_len = mel.shape[1]
    window, beg, eot = 2 * n_ctx, sp["beg"], sp["eot"]
    n_max = min(max_tokens, hp["n_text_ctx"] // 2 - 4)
    init = [sp["sot"]] + ([sp["sot"] + 1, sp["transcribe"]] if sp["multilingual"] else [])
    past, segs, margin, seek = [], [], np.inf, 0
    while seek < n_len:
        _, ck, cv = om.encode(mel, n_ctx=n_ctx, mel_offset=seek, n_threads=n_threads)
        # whisper_full: n_take = min(n_text_ctx / 2, past size) tokens after <|prev|>
        prompt = ([sp["prev"]] + past[-(hp["n_text_ctx"] // 2):] if past else []) + init
        toks, m = ts_window_ref(om, ck, cv, prompt, n_max, n_threads)
        margin = min(margin, m)
        seek_delta, result_len, failed, ended = window, 0, False, False
        for i, t in enumerate(toks):
            if t["id"] > beg:
                seek_delta, result_len = 2 * (t["id"] - beg), i + 1
            if t["id"] == eot:
                ended = True
                if result_len == 0:
                    if seek + seek_delta + 100 >= n_len:
                        result_len = i + 1
                    else:
                        failed = True
                break
        if not ended and (result_len == 0 or seek_delta < window // 2):
            failed = True
        if failed:
            seek += 100
            continue
        toks = toks[:result_len]
        past += [t["id"] for t in toks]
        if toks:
            i0, t0, text, i = 0, seek + 2 * (toks[0]["tid"] - beg), b"", 0
            while i < len(toks):
                if toks[i]["id"] < eot:
                    text += token_text(toks[i]["id"])
                if toks[i]["id"] > beg:
                    t1 = seek + 2 * (toks[i]["tid"] - beg)
                    if text:
                        segs.append({"t0": t0, "t1": t1, "text": text, "ids": [t["id"] for t in toks[i0:i + 1]]})
                    text = b""
                    while i < len(toks) and toks[i]["id"] > beg:
                        i += 1
                    i -= 1
                    t0, i0 = t1, i + 1
                i += 1
            if text:
                segs.append({"t0": t0, "t1": seek + seek_delta, "text": text, "ids": [t["id"] for t in toks[i0:]]})
        seek += seek_delta
    return segs, margin
