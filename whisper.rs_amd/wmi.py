"""Python mirror of the reference's pipeline interface over the C ABI.

The reference (szuwgh/whisper.rs, src/main.rs) exposes

    WhisperContext::new(fname) -> WsResult<WhisperContext>          main.rs:366
    whisper_pcm_to_mel(&mut ctx, samples: Arc<Vec<f32>>)            main.rs:1681
    whisper_encode(&mut ctx, n_threads, mel_offset)                 main.rs:1799
    convert_integer_to_float_audio(&[i16]) -> Vec<f32>              main.rs:1673
    WsError (BadMagic, UnknownTensor, WrongSizeTensor, ...)         main.rs:51-72

This module keeps those names, argument meanings and error behaviour, and
binds them with ctypes to libwhisper_mi355x.so (include/whisper_mi355x.h),
whose work runs in hand-written gfx950 kernels.  There is no CPU fallback:
if the shared library or a HIP device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WMI_LIB") or os.path.join(HERE, "libwhisper_mi355x.so")

WMI_OK = 0


class WsError(RuntimeError):
    """WsError (main.rs:51-72); `code` is the wmi_status value."""
    code = -1

    def __init__(self, msg: str = "", code: int | None = None):
        super().__init__(msg)
        if code is not None:
            self.code = code


class UnexpectIO(WsError): code = 1
class BadMagic(WsError): code = 2
class NotEnoughSpace(WsError): code = 3
class UnknownTensor(WsError): code = 4
class BadRefTensor(WsError): code = 5
class WrongSizeTensor(WsError): code = 6
class WrongShapeTensor(WsError): code = 7
class WrongBytesTensor(WsError): code = 8
class WrongGTensor(WsError): code = 9
class Unexpected(WsError): code = 10
class HipError(WsError): code = 11
class RcclError(WsError): code = 12
class Unsupported(WsError): code = 13
class InvalidArgument(WsError): code = 14


_ERRORS = {c.code: c for c in (UnexpectIO, BadMagic, NotEnoughSpace, UnknownTensor, BadRefTensor, WrongSizeTensor,
                               WrongShapeTensor, WrongBytesTensor, WrongGTensor, Unexpected, HipError, RcclError,
                               Unsupported, InvalidArgument)}

# exported symbols of include/whisper_mi355x.h
EXPORTS = (
    "wmi_init_from_file", "wmi_free", "wmi_strerror", "wmi_last_error", "wmi_last_error_global",
    "wmi_get_hparams", "wmi_get_special_tokens", "wmi_set_audio_ctx", "wmi_token_to_bytes",
    "wmi_read_wav", "wmi_pcm16_to_f32", "wmi_tokens_to_text",
    "wmi_decode_timestamps", "wmi_transcribe", "wmi_get_segment", "wmi_get_segment_tokens",
    "wmi_pcm_to_mel", "wmi_pcm_to_mel_batch", "wmi_encode", "wmi_decode_greedy", "wmi_decode_logits",
    "wmi_decode_beam", "wmi_full", "wmi_stage_pcm", "wmi_run_staged", "wmi_run_staged_beam", "wmi_get_tokens", "wmi_get_timings", "wmi_sync",
    "wmi_get_mel", "wmi_get_checksums", "wmi_get_encoder_out", "wmi_get_cross_kv", "wmi_bench_kernel", "wmi_decode_alg_bytes",
    "wmi_selftest", "wmi_debug_read",
    "wmi_dist_id_size", "wmi_dist_make_id", "wmi_dist_init", "wmi_dist_gather_tokens", "wmi_dist_barrier",
)


class Hparams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                                         "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer", "n_mels", "f16")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class SpecialTokens(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("eot", "sot", "prev", "solm", "not_", "beg", "translate", "transcribe",
                                         "is_multilingual")]


class KernelBench(C.Structure):
    _fields_ = [("avg_us", C.c_float), ("alg_bytes", C.c_double), ("alg_flops", C.c_double),
                ("name", C.c_char * 48)]


class TokenData(C.Structure):
    """WhisperTokenData (main.rs:317-331)."""
    _fields_ = [("id", C.c_int32), ("tid", C.c_int32), ("p", C.c_float), ("pt", C.c_float), ("ptsum", C.c_float),
                ("t0", C.c_int64), ("t1", C.c_int64), ("vlen", C.c_float)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Timings(C.Structure):
    _fields_ = [("mel_ms", C.c_float), ("encode_ms", C.c_float), ("cross_kv_ms", C.c_float),
                ("decode_ms", C.c_float), ("n_decode_steps", C.c_int32)]


_lib = None


def lib():
    """Load the HIP library (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        vp, i32, sz = C.c_void_p, C.c_int32, C.c_size_t
        L.wmi_init_from_file.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(vp)]
        L.wmi_free.argtypes = [vp]
        L.wmi_free.restype = None
        L.wmi_strerror.restype = C.c_char_p
        L.wmi_last_error.argtypes = [vp]
        L.wmi_last_error.restype = C.c_char_p
        L.wmi_last_error_global.restype = C.c_char_p
        L.wmi_get_hparams.argtypes = [vp, C.POINTER(Hparams)]
        L.wmi_get_special_tokens.argtypes = [vp, C.POINTER(SpecialTokens)]
        L.wmi_set_audio_ctx.argtypes = [vp, C.c_int]
        L.wmi_token_to_bytes.argtypes = [vp, i32, C.c_char_p, sz, C.POINTER(sz)]
        L.wmi_read_wav.argtypes = [C.c_char_p, vp, sz, C.POINTER(sz), C.POINTER(i32), C.POINTER(i32)]
        L.wmi_pcm16_to_f32.argtypes = [vp, sz, vp]
        L.wmi_tokens_to_text.argtypes = [vp, vp, C.c_int, C.c_char_p, sz, C.POINTER(sz)]
        L.wmi_decode_timestamps.argtypes = [vp, vp, C.c_int, C.c_int, vp, C.POINTER(i32)]
        L.wmi_transcribe.argtypes = [vp, vp, sz, C.c_int, C.POINTER(i32)]
        L.wmi_get_segment.argtypes = [vp, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_char_p, sz,
                                      C.POINTER(sz)]
        L.wmi_get_segment_tokens.argtypes = [vp, C.c_int, vp, sz, C.POINTER(i32)]
        L.wmi_pcm_to_mel.argtypes = [vp, vp, sz]
        L.wmi_pcm_to_mel_batch.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(sz)]
        L.wmi_stage_pcm.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(sz)]
        L.wmi_encode.argtypes = [vp, C.c_int, C.c_int]
        L.wmi_decode_greedy.argtypes = [vp, C.c_int, C.c_int, vp, vp]
        L.wmi_decode_logits.argtypes = [vp, C.c_int, vp, C.c_int, vp]
        L.wmi_full.argtypes = [vp, vp, sz, C.c_int, vp, vp]
        L.wmi_run_staged.argtypes = [vp, C.c_int, C.c_int]
        L.wmi_run_staged_beam.argtypes = [vp, C.c_int, C.c_int, C.c_int]
        L.wmi_decode_beam.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, vp, vp]
        L.wmi_get_tokens.argtypes = [vp, vp, sz, vp]
        L.wmi_get_timings.argtypes = [vp, C.POINTER(Timings)]
        L.wmi_sync.argtypes = [vp]
        L.wmi_get_mel.argtypes = [vp, C.c_int, vp, sz, C.POINTER(i32), C.POINTER(i32)]
        L.wmi_get_encoder_out.argtypes = [vp, C.c_int, vp, sz]
        L.wmi_get_cross_kv.argtypes = [vp, C.c_int, vp, vp, sz]
        L.wmi_bench_kernel.argtypes = [vp, C.c_int, C.c_int, C.POINTER(KernelBench)]
        L.wmi_decode_alg_bytes.argtypes = [C.POINTER(Hparams), C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.wmi_selftest.argtypes = [vp, C.POINTER(i32)]
        L.wmi_debug_read.argtypes = [vp, C.c_int, vp, C.c_size_t]
        L.wmi_get_checksums.argtypes = [vp, vp]
        L.wmi_dist_id_size.restype = sz
        L.wmi_dist_make_id.argtypes = [vp]
        L.wmi_dist_init.argtypes = [vp, C.c_int, C.c_int, vp]
        L.wmi_dist_gather_tokens.argtypes = [vp, vp, sz]
        L.wmi_dist_barrier.argtypes = [vp]
        _lib = L
    return _lib


def _raise(rc: int, ctx=None):
    if rc == WMI_OK:
        return
    L = lib()
    msg = (L.wmi_last_error(ctx) if ctx else L.wmi_last_error_global()) or b""
    cls = _ERRORS.get(rc, WsError)
    raise cls(f"{L.wmi_strerror(rc).decode()}: {msg.decode(errors='replace')}", rc)


def decode_alg_bytes(hp: dict, rows: int, steps: int, beam: bool = False, q5: bool = False):
    """(bytes, flops) of one decode (wmi_decode_alg_bytes: host-only, no device)."""
    h = Hparams(**{n: int(hp.get(n, 1)) for n, _ in Hparams._fields_})
    b, f = C.c_double(), C.c_double()
    _raise(lib().wmi_decode_alg_bytes(C.byref(h), rows, steps, int(bool(beam)), int(bool(q5)), C.byref(b),
                                      C.byref(f)))
    return b.value, f.value


def convert_integer_to_float_audio(samples) -> np.ndarray:
    """main.rs:1673-1679: s16 -> f32 / 32768.0."""
    return (np.asarray(samples, dtype=np.int16).astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def read_wav(path: str):
    """hound::WavReader::open + samples::<i16>() (main.rs:2067-2068) through
    the C ABI: (int16 samples interleaved, sample_rate, channels)."""
    L = lib()
    n, sr, ch = C.c_size_t(), C.c_int32(), C.c_int32()
    _raise(L.wmi_read_wav(os.fsencode(path), None, 0, C.byref(n), C.byref(sr), C.byref(ch)))
    out = np.zeros(n.value, np.int16)
    _raise(L.wmi_read_wav(os.fsencode(path), _ptr(out), out.size, C.byref(n), C.byref(sr), C.byref(ch)))
    return out, sr.value, ch.value


def pcm16_to_f32(s16) -> np.ndarray:
    """convert_integer_to_float_audio (main.rs:1673-1679) through the C ABI."""
    s16 = np.ascontiguousarray(s16, dtype=np.int16)
    out = np.zeros(s16.size, np.float32)
    _raise(lib().wmi_pcm16_to_f32(_ptr(s16), s16.size, _ptr(out)))
    return out


class WhisperContext:
    """WhisperContext (main.rs:333-363), device-resident."""

    def __init__(self, handle, device: int, max_clips: int):
        self._h = handle
        self.device = device
        self.max_clips = max_clips
        hp = Hparams()
        _raise(lib().wmi_get_hparams(self._h, C.byref(hp)), self._h)
        self.hparams = hp.as_dict()
        sp = SpecialTokens()
        _raise(lib().wmi_get_special_tokens(self._h, C.byref(sp)), self._h)
        self.special = {"eot": sp.eot, "sot": sp.sot, "prev": sp.prev, "solm": sp.solm, "not": sp.not_,
                        "beg": sp.beg, "translate": sp.translate, "transcribe": sp.transcribe,
                        "multilingual": sp.is_multilingual}
        self.n_clips = 0
        self.n_ctx = self.hparams["n_audio_ctx"]

    @classmethod
    def new(cls, fname: str, device: int = 0, max_clips: int = 1) -> "WhisperContext":
        """WhisperContext::new (main.rs:366-503); raises the WsError variant."""
        h = C.c_void_p()
        rc = lib().wmi_init_from_file(os.fsencode(fname), device, max_clips, C.byref(h))
        _raise(rc)
        return cls(h, device, max_clips)

    def close(self):
        if getattr(self, "_h", None):
            lib().wmi_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # --- knobs -------------------------------------------------------------
    def set_audio_ctx(self, n: int) -> None:
        """exp_n_audio_ctx (main.rs:362, 1803-1807); 0 restores n_audio_ctx."""
        _raise(lib().wmi_set_audio_ctx(self._h, n), self._h)
        self.n_ctx = n or self.hparams["n_audio_ctx"]

    def token_to_str(self, tid: int) -> bytes:
        """id_to_token (main.rs:578-592, 442-467)."""
        n = C.c_size_t()
        buf = C.create_string_buffer(512)
        _raise(lib().wmi_token_to_bytes(self._h, tid, buf, 512, C.byref(n)), self._h)
        return buf.raw[:n.value]

    def tokens_to_text(self, ids) -> bytes:
        """Text bytes of the text tokens of ids (specials / timestamps skipped)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        n = C.c_size_t()
        rc = lib().wmi_tokens_to_text(self._h, _ptr(ids), ids.size, None, 0, C.byref(n))
        if rc not in (WMI_OK, NotEnoughSpace.code):
            _raise(rc, self._h)
        buf = C.create_string_buffer(max(1, n.value))
        _raise(lib().wmi_tokens_to_text(self._h, _ptr(ids), ids.size, buf, n.value, C.byref(n)), self._h)
        return buf.raw[:n.value]

    # --- timestamps / segments (whisper.cpp-1.0.3 whisper_full) ----------
    def decode_timestamps(self, prompt, max_tokens: int):
        """One timestamp-decoding window of encoded clip 0: [WhisperTokenData dict]."""
        prompt = np.ascontiguousarray(prompt, dtype=np.int32)
        out = (TokenData * max_tokens)()
        n = C.c_int32()
        _raise(lib().wmi_decode_timestamps(self._h, _ptr(prompt), prompt.size, max_tokens, out, C.byref(n)), self._h)
        return [out[i].as_dict() for i in range(n.value)]

    def transcribe(self, pcm, max_tokens: int = 220):
        """whisper_full with timestamps: [{"t0", "t1", "text", "tokens"}] (t in 10 ms)."""
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        ns = C.c_int32()
        _raise(lib().wmi_transcribe(self._h, _ptr(pcm), pcm.size, max_tokens, C.byref(ns)), self._h)
        self.n_clips = 1
        segs = []
        for i in range(ns.value):
            t0, t1, ln = C.c_int64(), C.c_int64(), C.c_size_t()
            lib().wmi_get_segment(self._h, i, C.byref(t0), C.byref(t1), None, 0, C.byref(ln))
            buf = C.create_string_buffer(max(1, ln.value))
            _raise(lib().wmi_get_segment(self._h, i, C.byref(t0), C.byref(t1), buf, ln.value, C.byref(ln)), self._h)
            nt = C.c_int32()
            lib().wmi_get_segment_tokens(self._h, i, None, 0, C.byref(nt))
            toks = (TokenData * max(1, nt.value))()
            _raise(lib().wmi_get_segment_tokens(self._h, i, toks, nt.value, C.byref(nt)), self._h)
            segs.append({"t0": t0.value, "t1": t1.value, "text": buf.raw[:ln.value],
                         "tokens": [toks[k].as_dict() for k in range(nt.value)]})
        return segs

    # --- pipeline ---------------------------------------------------------
    def pcm_to_mel_batch(self, clips) -> None:
        clips = [np.ascontiguousarray(c, dtype=np.float32) for c in clips]
        ptrs = (C.c_void_p * len(clips))(*[c.ctypes.data for c in clips])
        ns = (C.c_size_t * len(clips))(*[c.size for c in clips])
        _raise(lib().wmi_pcm_to_mel_batch(self._h, len(clips), ptrs, ns), self._h)
        self.n_clips = len(clips)

    def encode(self, n_threads: int = 1, mel_offset: int = 0) -> None:
        _raise(lib().wmi_encode(self._h, n_threads, mel_offset), self._h)

    def decode_greedy(self, max_tokens: int, suppress_eot: bool = False):
        toks = np.zeros((self.n_clips, max_tokens), np.int32)
        cnt = np.zeros(self.n_clips, np.int32)
        _raise(lib().wmi_decode_greedy(self._h, max_tokens, int(suppress_eot), _ptr(toks), _ptr(cnt)), self._h)
        return [toks[i, :cnt[i]].copy() for i in range(self.n_clips)]

    def decode_beam(self, beam_size: int, max_tokens: int, suppress_eot: bool = False):
        """Beam search per clip: [(tokens, score)] (semantics: oracle/wmi_oracle.h)."""
        toks = np.zeros((self.n_clips, max_tokens), np.int32)
        cnt = np.zeros(self.n_clips, np.int32)
        sc = np.zeros(self.n_clips, np.float64)
        _raise(lib().wmi_decode_beam(self._h, beam_size, max_tokens, int(suppress_eot), _ptr(toks), _ptr(cnt),
                                     _ptr(sc)), self._h)
        return [(toks[i, :cnt[i]].copy(), float(sc[i])) for i in range(self.n_clips)]

    def decode_logits(self, tokens, clip: int = 0) -> np.ndarray:
        tokens = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.zeros((tokens.size, self.hparams["n_vocab"]), np.float32)
        _raise(lib().wmi_decode_logits(self._h, clip, _ptr(tokens), tokens.size, _ptr(out)), self._h)
        return out

    def full(self, pcm, max_tokens: int = 224) -> np.ndarray:
        """Transcribe: pcm_to_mel -> encode -> greedy decode (token ids)."""
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        toks = np.zeros(max_tokens, np.int32)
        cnt = np.zeros(1, np.int32)
        _raise(lib().wmi_full(self._h, _ptr(pcm), pcm.size, max_tokens, _ptr(toks), _ptr(cnt)), self._h)
        self.n_clips = 1
        return toks[:cnt[0]].copy()

    def stage(self, clips) -> None:
        clips = [np.ascontiguousarray(c, dtype=np.float32) for c in clips]
        ptrs = (C.c_void_p * len(clips))(*[c.ctypes.data for c in clips])
        ns = (C.c_size_t * len(clips))(*[c.size for c in clips])
        _raise(lib().wmi_stage_pcm(self._h, len(clips), ptrs, ns), self._h)
        self.n_clips = len(clips)

    def run_staged(self, n_decode: int = 128, mel_offset: int = 0, beam_size: int = 0) -> None:
        _raise(lib().wmi_run_staged_beam(self._h, mel_offset, n_decode, beam_size), self._h)
        self._n_decode = n_decode

    def tokens(self) -> np.ndarray:
        out = np.zeros((self.n_clips, self._n_decode), np.int32)
        _raise(lib().wmi_get_tokens(self._h, _ptr(out), out.size, None), self._h)
        return out

    def timings(self) -> dict:
        t = Timings()
        _raise(lib().wmi_get_timings(self._h, C.byref(t)), self._h)
        return {"mel_ms": t.mel_ms, "encode_ms": t.encode_ms, "cross_kv_ms": t.cross_kv_ms,
                "decode_ms": t.decode_ms, "n_decode_steps": t.n_decode_steps}

    def bench_kernel(self, which: int, iters: int = 50) -> dict:
        """Mean duration of one kernel of the last run (HIP events, same stream)."""
        kb = KernelBench()
        _raise(lib().wmi_bench_kernel(self._h, which, iters, C.byref(kb)), self._h)
        return {"name": kb.name.decode(), "avg_us": kb.avg_us, "alg_bytes": kb.alg_bytes, "alg_flops": kb.alg_flops}

    def selftest(self) -> int:
        """Mismatches of the device-computed f16 exp vs the host ggml table."""
        n = C.c_int32()
        _raise(lib().wmi_selftest(self._h, C.byref(n)), self._h)
        return n.value

    def checksums(self) -> dict:
        """The reference's stage sums (wmi_get_checksums; WMI_CHECKSUMS=1 contexts)."""
        out = np.zeros(5, np.float32)
        _raise(lib().wmi_get_checksums(self._h, _ptr(out)), self._h)
        return dict(zip(("hann", "samples", "filters", "mel_raw", "mel_window"), out.tolist()))

    def debug_read(self, which: int, nbytes: int) -> bytes:
        """Raw copy of a device buffer of the last decode (wmi_debug_read)."""
        buf = C.create_string_buffer(nbytes)
        _raise(lib().wmi_debug_read(self._h, which, buf, nbytes), self._h)
        return buf.raw

    def step_logits(self, n_pos: int) -> np.ndarray:
        """Every position's logits of the last persistent greedy decode or
        beam search, [n_pos][rows][V] with rows = max(8, max_clips) (contexts
        created with WMI_LOGITS_ALL=1: position p's logits predict the token
        after the one fed at p; greedy: clip b in row b; beam: slot s)."""
        V = self.hparams["n_vocab"]
        rows = int(np.frombuffer(self.debug_read(16, 4), np.int32)[0])
        raw = self.debug_read(13, n_pos * rows * V * 4)
        return np.frombuffer(raw, np.float32).reshape(n_pos, rows, V).copy()

    def beam_history(self, n_steps: int):
        """The last beam search's selections (its last clip): (parent slot,
        token) arrays [n_steps][8] — slot s after generation step t came from
        slot parent[t][s] of step t - 1 and appended token[t][s]."""
        par = np.frombuffer(self.debug_read(14, n_steps * 8 * 4), np.int32).reshape(n_steps, 8).copy()
        tok = np.frombuffer(self.debug_read(15, n_steps * 8 * 4), np.int32).reshape(n_steps, 8).copy()
        return par, tok

    # --- parity getters -----------------------------------------------------
    def mel(self, clip: int = 0) -> np.ndarray:
        nm, nl = C.c_int32(), C.c_int32()
        _raise(lib().wmi_get_mel(self._h, clip, None, 0, C.byref(nm), C.byref(nl)), self._h)
        out = np.zeros((nm.value, nl.value), np.float32)
        _raise(lib().wmi_get_mel(self._h, clip, _ptr(out), out.size, C.byref(nm), C.byref(nl)), self._h)
        return out

    def encoder_out(self, clip: int = 0) -> np.ndarray:
        out = np.zeros((self.n_ctx, self.hparams["n_audio_state"]), np.float32)
        _raise(lib().wmi_get_encoder_out(self._h, clip, _ptr(out), out.size), self._h)
        return out

    def cross_kv(self, clip: int = 0):
        shp = (self.hparams["n_text_layer"], self.n_ctx, self.hparams["n_text_state"])
        k = np.zeros(shp, np.uint16)
        v = np.zeros(shp, np.uint16)
        _raise(lib().wmi_get_cross_kv(self._h, clip, _ptr(k), _ptr(v), k.size), self._h)
        return k, v

    # --- multi-GPU ----------------------------------------------------------
    @staticmethod
    def dist_make_id() -> bytes:
        n = lib().wmi_dist_id_size()
        buf = C.create_string_buffer(n)
        _raise(lib().wmi_dist_make_id(buf))
        return buf.raw

    def dist_init(self, rank: int, world: int, uid: bytes) -> None:
        buf = C.create_string_buffer(uid, len(uid))
        _raise(lib().wmi_dist_init(self._h, rank, world, buf), self._h)
        self.rank, self.world = rank, world

    def dist_gather_tokens(self):
        """Root: (tokens [world][clips][n_decode] with -1 padding, counts
        [world][clips]); other ranks: None."""
        rec = self._n_decode + 1
        total = self.world * self.n_clips * rec
        out = np.zeros(total, np.int32) if self.rank == 0 else None
        _raise(lib().wmi_dist_gather_tokens(self._h, _ptr(out) if out is not None else None, total), self._h)
        if out is None:
            return None
        blk = out.reshape(self.world, self.n_clips, rec)
        return blk[:, :, 1:].copy(), blk[:, :, 0].copy()

    def dist_barrier(self) -> None:
        _raise(lib().wmi_dist_barrier(self._h), self._h)


# reference-named free functions -----------------------------------------------
def whisper_pcm_to_mel(ctx: WhisperContext, samples) -> None:
    """main.rs:1681-1707."""
    ctx.pcm_to_mel_batch([samples])


def whisper_encode(ctx: WhisperContext, n_threads: int, mel_offset: int) -> None:
    """main.rs:1799-2063 (n_threads accepted and ignored, as in the reference)."""
    ctx.encode(n_threads, mel_offset)
