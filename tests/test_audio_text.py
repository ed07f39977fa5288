"""WAV input and text output through the C ABI.

The reference reads its audio with hound (main.rs:2067-2068:
WavReader::open(path).samples::<i16>()) and converts it with
convert_integer_to_float_audio (main.rs:1673-1679); wmi_read_wav /
wmi_pcm16_to_f32 replace both and need no device, so they run here.  The
detokeniser (id_to_token bytes, main.rs:578-592, text tokens only) needs a
context, hence a GPU box.
"""
import os
import struct

import numpy as np
import pytest

import synth
import wmi


def _wav(path, payload: bytes, fmt_tag=1, ch=1, sr=16000, bits=16, extra_chunk=b""):
    with open(path, "wb") as f:
        body = b"WAVE" + b"fmt " + struct.pack("<IHHIIHH", 16, fmt_tag, ch, sr, sr * ch * bits // 8, ch * bits // 8, bits)
        body += extra_chunk + b"data" + struct.pack("<I", len(payload)) + payload
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_read_wav_roundtrip_matches_reference_conversion(tmp_path):
    s16 = synth.synth_pcm_i16(1.5, 77)
    path = os.path.join(str(tmp_path), "clip.wav")
    synth.write_wav(path, s16)
    got, sr, ch = wmi.read_wav(path)
    assert (sr, ch) == (16000, 1)
    np.testing.assert_array_equal(got, s16)
    # the product conversion equals the reference expression s / 32768.0 (f32)
    np.testing.assert_array_equal(wmi.pcm16_to_f32(got), wmi.convert_integer_to_float_audio(s16))
    np.testing.assert_array_equal(wmi.pcm16_to_f32(got), synth.pcm_i16_to_f32(s16))


def test_read_wav_stereo_and_skipped_chunks(tmp_path):
    inter = np.arange(-500, 500, dtype=np.int16)  # 500 stereo frames, interleaved
    path = os.path.join(str(tmp_path), "st.wav")
    odd_chunk = b"LIST" + struct.pack("<I", 3) + b"abc" + b"\x00"  # odd size: padded to a word
    _wav(path, inter.astype("<i2").tobytes(), ch=2, sr=44100, extra_chunk=odd_chunk)
    got, sr, ch = wmi.read_wav(path)
    assert (sr, ch) == (44100, 2)
    np.testing.assert_array_equal(got, inter)


def test_read_wav_errors(tmp_path):
    d = str(tmp_path)
    with pytest.raises(wmi.UnexpectIO):
        wmi.read_wav(os.path.join(d, "missing.wav"))
    bad = os.path.join(d, "bad.wav")
    open(bad, "wb").write(b"RIFX" + b"\x00" * 40)
    with pytest.raises(wmi.UnexpectIO):
        wmi.read_wav(bad)
    f32 = os.path.join(d, "float.wav")
    _wav(f32, np.zeros(8, "<f4").tobytes(), fmt_tag=3, bits=32)
    with pytest.raises(wmi.Unsupported):
        wmi.read_wav(f32)
    trunc = os.path.join(d, "trunc.wav")
    synth.write_wav(trunc, np.arange(100, dtype=np.int16))
    open(trunc, "r+b").truncate(44 + 50)
    with pytest.raises(wmi.UnexpectIO):
        wmi.read_wav(trunc)


def test_read_wav_empty_data(tmp_path):
    path = os.path.join(str(tmp_path), "empty.wav")
    synth.write_wav(path, np.zeros(0, np.int16))
    got, sr, ch = wmi.read_wav(path)
    assert got.size == 0 and sr == 16000 and ch == 1


@pytest.mark.gpu
def test_tokens_to_text(micro_model):
    ctx = wmi.WhisperContext.new(micro_model, 0, max_clips=1)
    try:
        sp = ctx.special
        ids = [sp["sot"], 3, 17, sp["beg"] + 5, 250, sp["eot"]]
        want = b"".join(ctx.token_to_str(i) for i in (3, 17, 250))
        assert ctx.tokens_to_text(ids) == want
        assert ctx.tokens_to_text([]) == b""
        with pytest.raises(wmi.InvalidArgument):
            ctx.tokens_to_text([ctx.hparams["n_vocab"]])
    finally:
        ctx.close()
