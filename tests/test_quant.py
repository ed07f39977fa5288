"""ggml quantised weight files.

The reference loader rejects quantised tensors (main.rs:1423-1434); this
build dequantises every quantised matrix to f16, w = f16(q * d (+ m)) rounded
once, as a fused multiply-add (ggml's GPU back-ends' dequantise -> f16 GEMM),
so every matmul keeps the f16 semantics of SURVEY.md §A.4.  Pinned here: the
synthetic quantisers restate ggml's quantize_row_*_ref, and the oracle's
dequantisation equals an independent NumPy decoding of the QNT-v2 block
layouts bit for bit.  CPU only.
"""
import os

import numpy as np
import pytest

import pyoracle
import synth

TYPES = {"q4_0": (2, 18), "q4_1": (3, 20), "q5_0": (6, 22), "q5_1": (7, 24), "q8_0": (8, 34)}


def np_dequant(qtype: str, raw: bytes, nel: int) -> np.ndarray:
    """Independent decoding of ggml QNT-v2 blocks -> f16 (as float32 values)."""
    nb = nel // 32
    b = np.frombuffer(raw, np.uint8).reshape(nb, TYPES[qtype][1])
    d = b[:, 0:2].copy().view("<f2")[:, 0].astype(np.float32)
    if qtype == "q8_0":
        q = b[:, 2:34].view(np.int8).astype(np.int32)
        return (q.astype(np.float64) * d[:, None]).astype(np.float16).reshape(-1)
    m = b[:, 2:4].copy().view("<f2")[:, 0].astype(np.float32) if qtype in ("q4_1", "q5_1") else None
    qs_off = {"q4_0": 2, "q4_1": 4, "q5_0": 6, "q5_1": 8}[qtype]
    qs = b[:, qs_off:qs_off + 16].astype(np.int32)
    q = np.concatenate([qs & 15, qs >> 4], axis=1)
    if qtype in ("q5_0", "q5_1"):
        ho = 2 if qtype == "q5_0" else 4
        qh = b[:, ho:ho + 4].copy().view("<u4")[:, 0].astype(np.int64)
        q = q | (((qh[:, None] >> np.arange(32)) & 1) << 4).astype(np.int32)
    off = {"q4_0": 8, "q5_0": 16}.get(qtype, 0)
    v = (q - off).astype(np.float64) * d[:, None].astype(np.float64)  # exact
    if m is not None:
        v = v + m[:, None].astype(np.float64)  # exact for these magnitudes
    return v.astype(np.float16).reshape(-1)  # one RNE rounding (NumPy rounds double -> half directly)


@pytest.mark.parametrize("qtype", sorted(TYPES))
def test_quantiser_and_oracle_dequant(qtype):
    rng = np.random.default_rng(5)
    w = (rng.standard_normal((64, 128)) * 0.02).astype(np.float16).astype(np.float32)
    w[3, :32] = 0.0  # an all-zero block (d = 0)
    raw = synth.quantize(w, qtype)
    assert len(raw) == w.size // 32 * TYPES[qtype][1]
    ref = np_dequant(qtype, raw, w.size)
    got = pyoracle.dequant(TYPES[qtype][0], raw, w.size).view(np.float16)
    np.testing.assert_array_equal(got.view(np.uint16), ref.view(np.uint16))
    bits = {"q4_0": 4, "q4_1": 4, "q5_0": 5, "q5_1": 5, "q8_0": 8}[qtype]
    span = np.abs(w).max() * 2
    assert np.abs(got.astype(np.float32).reshape(w.shape) - w).max() <= span / (2 ** bits - 1) + 1e-3
    assert np.all(got.reshape(64, 128)[3, :32] == 0)


@pytest.mark.parametrize("qtype", ["q5_1", "q8_0"])
def test_quantised_file_loads(model_cache, qtype):
    path = os.path.join(model_cache, f"ggml-synth-micro-{qtype}.bin")
    if not os.path.exists(path):
        synth.write_ggml(path, "micro", quant=qtype)
    om = pyoracle.OracleModel(path)
    assert om.hp["f16"] == synth.QUANT_TYPES[qtype][1] + 1000 * synth.GGML_QNT_VERSION
    om.close()


def test_unsupported_quant_version(tmp_path):
    path = str(tmp_path / "v1.bin")
    synth.write_ggml(path, "micro", quant="q5_1", hp_override={})
    raw = bytearray(open(path, "rb").read())
    import struct
    raw[4 + 40:4 + 44] = struct.pack("<i", 1009)  # QNT version 1
    open(path, "wb").write(raw)
    with pytest.raises(pyoracle.OracleError) as e:
        pyoracle.OracleModel(path)
    assert e.value.code == 13


@pytest.mark.parametrize("qtype", sorted(TYPES))
def test_dequant_rounding_random_blocks(qtype):
    """Arbitrary blocks (random quants, d and m over f16's whole normal and
    subnormal exponent range): the single-rounding dequantisation equals
    NumPy's correctly rounded double -> half conversion everywhere."""
    rng = np.random.default_rng(11)
    nb, bs = 2048, TYPES[qtype][1]
    raw = rng.integers(0, 256, (nb, bs), dtype=np.uint8)
    e = rng.integers(-24, 8, (nb, 2))
    vals = (rng.choice([-1.0, 1.0], (nb, 2)) * rng.uniform(1, 2, (nb, 2)) * np.exp2(e)).astype(np.float16)
    raw[:, 0:2] = vals[:, 0:1].copy().view(np.uint8)
    if qtype in ("q4_1", "q5_1"):
        raw[:, 2:4] = vals[:, 1:2].copy().view(np.uint8)
    raw = raw.tobytes()
    ref = np_dequant(qtype, raw, nb * 32)
    got = pyoracle.dequant(TYPES[qtype][0], raw, nb * 32)
    np.testing.assert_array_equal(got, ref.view(np.uint16))


@pytest.mark.parametrize("hook", ["sharp_hook", "xsharp_hook", "xsharp_lv3_hook", "lnmean_hook"])
def test_derived_variant_equals_generated(tmp_path, hook):
    """synth.derive_variant (a copy of the plain file with the hooked tensors
    rewritten) gives byte for byte the file write_ggml writes with the hook."""
    import synth
    plain, gen, der = (str(tmp_path / n) for n in ("plain.bin", "gen.bin", "der.bin"))
    synth.write_ggml(plain, "micro")
    synth.write_ggml(gen, "micro", tensor_hook=getattr(synth, hook))
    synth.derive_variant(plain, der, getattr(synth, hook))
    with open(gen, "rb") as a, open(der, "rb") as b:
        assert a.read() == b.read()
