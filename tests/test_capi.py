"""CPU tests of the C ABI (libwhisper_mi355x.so): the library loads, exports
every entry point include/whisper_mi355x.h declares, and reproduces the
reference loader's error behaviour (WsError variants and their order,
main.rs:1384-1475) on malformed files — the file is parsed before any device
is touched, so these run without a GPU.  No compute is called here.
"""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

import pyoracle
import synth
import wmi
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "whisper_mi355x.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(wmi_[a-z_0-9]+)\s*\(", src, re.M)))


def test_header_exports_match_library():
    declared = header_functions()
    assert len(declared) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", wmi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (wmi_[a-z_0-9]+)$", out, re.M))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(wmi.EXPORTS) == declared
    lib = wmi.lib()
    for f in declared:
        assert getattr(lib, f) is not None


def test_strerror_covers_every_status():
    lib = wmi.lib()
    for code in range(0, 15):
        assert lib.wmi_strerror(code) not in (None, b"", b"unknown status")
    assert lib.wmi_strerror(99) == b"unknown status"


# --- malformed model files --------------------------------------------------

def _write_variant(tmp_path, name, mutate):
    """Write the micro model with one record mutated by `mutate(name, ne, ftype, payload)`."""
    path = os.path.join(tmp_path, name)
    hp = dict(synth.MODEL_DIMS["micro"], f16=1)
    with open(path, "wb") as f:
        f.write(struct.pack("<I", synth.GGML_MAGIC))
        f.write(struct.pack("<11i", *[hp[k] for k in synth.HPARAM_ORDER]))
        filt = synth.mel_filterbank(80)
        f.write(struct.pack("<ii", *filt.shape))
        f.write(filt.astype("<f4").tobytes())
        f.write(struct.pack("<i", 3))
        for tok in (b"a", b"b", b"c"):
            f.write(struct.pack("<I", len(tok)) + tok)
        for tname, shape, kind in synth.tensor_specs(hp):
            arr = synth.tensor_value(tname, shape, kind, hp)
            ftype = 1 if arr.dtype == np.float16 else 0
            ne = list(reversed(shape))
            payload = arr.astype("<f2" if ftype else "<f4").tobytes()
            r = mutate(tname, ne, ftype, payload)
            if r is None:
                continue
            tname, ne, ftype, payload = r
            nb = tname.encode()
            f.write(struct.pack("<iii", len(ne), len(nb), ftype))
            f.write(struct.pack(f"<{len(ne)}i", *ne))
            f.write(nb)
            f.write(payload)
    return path


CASES = {
    "unknown_tensor": (lambda n, ne, ft, p: ("encoder.bogus", ne, ft, p) if n == "encoder.conv1.bias" else (n, ne, ft, p),
                       wmi.UnknownTensor, 4),
    "wrong_size": (lambda n, ne, ft, p: (n, [ne[0] + 1] + ne[1:], ft, p) if n == "encoder.ln_post.bias" else (n, ne, ft, p),
                   wmi.WrongSizeTensor, 6),
    "wrong_shape": (lambda n, ne, ft, p: (n, list(reversed(ne)), ft, p)
                    if n == "encoder.blocks.0.mlp.0.weight" else (n, ne, ft, p), wmi.WrongShapeTensor, 7),
    "wrong_bytes": (lambda n, ne, ft, p: (n, ne, 1, p[: len(p) // 2]) if n == "encoder.ln_post.weight" else (n, ne, ft, p),
                    wmi.WrongBytesTensor, 8),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_loader_errors_match_reference_variants(tmp_path, case):
    mutate, exc, code = CASES[case]
    path = _write_variant(str(tmp_path), case + ".bin", mutate)
    with pytest.raises(exc) as ei:
        wmi.WhisperContext.new(path)
    assert ei.value.code == code
    with pytest.raises(pyoracle.OracleError) as oe:  # the oracle restates the same checks
        pyoracle.OracleModel(path)
    assert oe.value.code == code


def test_bad_magic_and_truncation(tmp_path, micro_model):
    bad = os.path.join(str(tmp_path), "bad.bin")
    data = open(micro_model, "rb").read()
    open(bad, "wb").write(b"ggjt" + data[4:])
    with pytest.raises(wmi.BadMagic):
        wmi.WhisperContext.new(bad)
    trunc = os.path.join(str(tmp_path), "trunc.bin")
    open(trunc, "wb").write(data[: len(data) - 1000])
    with pytest.raises(wmi.UnexpectIO):
        wmi.WhisperContext.new(trunc)
    with pytest.raises(wmi.UnexpectIO):
        wmi.WhisperContext.new(os.path.join(str(tmp_path), "does-not-exist.bin"))


def test_f32_model_parses(tmp_path):
    """ftype-0 files load (main.rs:817-821, 1423-1427: every matrix f32): the
    host parse passes and only device init remains; an f16 record in such a
    file is a wrong-bytes error, as in the reference's record loop."""
    path = _write_variant(str(tmp_path), "f32.bin",
                          lambda n, ne, ft, p: (n, ne, 0, np.frombuffer(p, "<f2").astype("<f4").tobytes()) if ft else (n, ne, ft, p))
    raw = bytearray(open(path, "rb").read())
    raw[4 + 40:4 + 44] = struct.pack("<i", 0)
    open(path, "wb").write(raw)
    try:
        wmi.WhisperContext.new(path).close()
    except wmi.HipError as e:
        assert "no HIP device" in str(e)
    pyoracle.OracleModel(path).close()
    mixed = os.path.join(str(tmp_path), "mixed.bin")
    data = open(_write_variant(str(tmp_path), "f16.bin", lambda *r: r), "rb").read()
    open(mixed, "wb").write(data[:44] + struct.pack("<i", 0) + data[48:])
    with pytest.raises(wmi.WrongBytesTensor):
        wmi.WhisperContext.new(mixed)


def test_valid_model_reaches_device_init(micro_model):
    """A valid file parses; the context then needs a HIP device and fails
    loudly without one (there is no CPU fallback)."""
    try:
        ctx = wmi.WhisperContext.new(micro_model)
    except wmi.HipError as e:
        assert "no HIP device" in str(e)
    else:  # on a GPU box
        assert ctx.hparams["n_audio_state"] == 128
        ctx.close()


def test_pcm_conversion_matches_reference():
    s16 = np.array([-32768, -1, 0, 1, 32767], np.int16)
    np.testing.assert_array_equal(wmi.convert_integer_to_float_audio(s16),
                                  np.array([-1.0, -1 / 32768, 0.0, 1 / 32768, 32767 / 32768], np.float32))


def test_hostile_headers_allocate_nothing(tmp_path, micro_model):
    """Header fields that would size huge host allocations are checked
    against the file first: out-of-range hparams, a vocabulary
    count or a WAV data chunk larger than the file — each a status code, not
    a std::bad_alloc escaping the C ABI."""
    data = open(micro_model, "rb").read()
    d = str(tmp_path)
    big = os.path.join(d, "hp.bin")  # n_vocab = 2^30
    open(big, "wb").write(data[:4] + struct.pack("<i", 1 << 30) + data[8:])
    with pytest.raises(wmi.Unexpected):
        wmi.WhisperContext.new(big)
    nfilt = struct.unpack("<ii", data[48:56])
    voc_off = 56 + 4 * nfilt[0] * nfilt[1]
    nv = os.path.join(d, "nv.bin")  # vocabulary of 2^31 - 1 entries in a small file
    open(nv, "wb").write(data[:voc_off] + struct.pack("<i", 0x7FFFFFFF) + data[voc_off + 4:])
    with pytest.raises(wmi.UnexpectIO):
        wmi.WhisperContext.new(nv)
    wav = os.path.join(d, "huge.wav")  # data chunk claims 4 GiB - 2
    body = b"WAVE" + b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, 16000, 32000, 2, 16)
    body += b"data" + struct.pack("<I", 0xFFFFFFFE) + b"\x00\x01" * 8
    open(wav, "wb").write(b"RIFF" + struct.pack("<I", len(body)) + body)
    with pytest.raises(wmi.UnexpectIO):
        wmi.read_wav(wav)


def test_decode_alg_bytes_counts_q5_blocks():
    """wmi_decode_alg_bytes (host only) is the one byte count of a decode:
    wmi_bench_kernel 14 reports it and bench.py's roofline uses it.  For a
    q5_1 decode the five GEMV matrices (13 n^2 weights) count at 24 bytes a
    32-weight block and Wcq stays f16: per layer and step 28 n^2 -> 11.75 n^2
    bytes; beam rows read their clip's cross K/V once."""
    import bench
    hp = dict(synth.MODEL_DIMS["small"], f16=1)
    n, L, T = hp["n_text_state"], hp["n_text_layer"], hp["n_audio_ctx"]
    steps = 131
    f16, fl = wmi.decode_alg_bytes(hp, 1, steps)
    q5, fl5 = wmi.decode_alg_bytes(hp, 1, steps, q5=True)
    assert fl == fl5 > 0
    assert f16 - q5 == pytest.approx(steps * L * (28.0 - 11.75) * n * n, rel=1e-12)
    # the bench leg of C3 charges exactly the library's q5_1 count (WMI_PERSIST_Q5 unset)
    old = os.environ.pop("WMI_PERSIST_Q5", None)
    try:
        assert bench.persist_q5("small-q5_1") and not bench.persist_q5("small")
        assert bench.decode_bytes(wmi, hp, 1, steps, False, bench.persist_q5("small-q5_1")) == q5
        assert bench.decode_bytes(wmi, hp, 5, steps, True, True) == wmi.decode_alg_bytes(hp, 5, steps, beam=True)[0]
    finally:
        if old is not None:
            os.environ["WMI_PERSIST_Q5"] = old
    b5, _ = wmi.decode_alg_bytes(hp, 5, steps, beam=True)
    g5, _ = wmi.decode_alg_bytes(hp, 5, steps)
    assert g5 - b5 == pytest.approx(steps * 4 * L * T * n * 4, rel=1e-12)  # 4 more clips' cross K/V
    with pytest.raises(wmi.InvalidArgument):
        wmi.decode_alg_bytes(hp, 0, steps)
