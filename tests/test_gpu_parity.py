"""HIP path vs the CPU restatement (oracle/), through the C ABI.

Tolerances (north_star "within 1e-3 on encoder activations"): max abs error
<= max(1e-3, 1.25 x the arithmetic's own noise floor) and mean abs error
<= max(3e-4, 1.25 x the floor's mean).  The noise floor is measured in the test: the same CPU restatement
run with exact (double) dot products instead of ggml's AVX2 f32 accumulation
order.  At base that floor is 1.34e-3 max / 1.9e-4 mean — an absolute 1e-3
bound is below what ANY reordering of the same f16/f32 arithmetic achieves
(DESIGN.md "Parity"); the HIP path sits at the floor.  Greedy
token ids bit-exact (a step whose oracle top-2 logit margin is below 1e-3 is
reported and excluded — a different f32 summation order may legitimately flip
such a near-tie); f16 outputs (cross K/V) within one f16 ulp.
Parity is against the restatement, which is itself "parity unpinned" with
respect to the reference (oracle/README.md).
"""
import numpy as np
import pytest

import pyoracle
import synth
from conftest import threads

pytestmark = pytest.mark.gpu

ENC_TOL = 1e-3


def f16(bits):
    return np.asarray(bits, np.uint16).view(np.float16).astype(np.float32)


def f16_ulp_ok(a_bits, b_bits, max_ulps=1):
    a, b = f16(a_bits), f16(b_bits)
    ulp = np.spacing(np.maximum(np.abs(a), np.abs(b)).astype(np.float16)).astype(np.float32)
    return np.abs(a - b) <= max_ulps * ulp + 1e-12


# The oracle's encoder outputs, memoised per (model file, clip, n_ctx,
# mel_offset, dot mode): the tests encode the same clips in several places
# (the floor needs a second, exact-dot encode), and a large-v3 encode takes
# tens of seconds of the box's 16 host threads.  Oldest entries dropped first.
_ENC_CACHE = {}
_ENC_CACHE_MAX = 16


def _oracle_encode(om, pcm, n_ctx, mel_offset=0, exact=False):
    """(enc [n_ctx][n], cross_k, cross_v) of the oracle for pcm; exact: with
    exact (double) dot products instead of ggml's order (the noise floor)."""
    import hashlib
    key = (om.path, hashlib.sha1(np.ascontiguousarray(pcm, np.float32).tobytes()).hexdigest(), n_ctx, mel_offset,
           exact)
    hit = _ENC_CACHE.pop(key, None)
    if hit is None:
        mel = om.mel(pcm, n_threads=threads())
        pyoracle.set_dot_mode(exact)
        try:
            hit = om.encode(mel, n_ctx=n_ctx, mel_offset=mel_offset, n_threads=threads())
        finally:
            pyoracle.set_dot_mode(False)
        while len(_ENC_CACHE) >= _ENC_CACHE_MAX:
            _ENC_CACHE.pop(next(iter(_ENC_CACHE)))
    _ENC_CACHE[key] = hit
    return hit


@pytest.fixture(scope="module")
def wmi():
    import wmi as w
    return w


@pytest.fixture(scope="module")
def micro_ctx(wmi, micro_model):
    ctx = wmi.WhisperContext.new(micro_model, 0, max_clips=4)
    yield ctx
    ctx.close()


def test_device_exp_matches_ggml_table(micro_ctx):
    """The decoder computes exp instead of reading ggml's f16 table: every one
    of the 31745 non-positive f16 inputs must give the table's exact entry."""
    assert micro_ctx.selftest() == 0


def test_mel_bit_parity(micro_ctx, oracle_micro):
    for secs, seed in ((2.0, 1234), (30.0, 7), (0.37, 3)):
        pcm = synth.synth_pcm_f32(secs, seed)
        ref = oracle_micro.mel(pcm, n_threads=threads())
        micro_ctx.pcm_to_mel_batch([pcm])
        got = micro_ctx.mel(0)
        assert got.shape == ref.shape
        d = np.abs(got - ref)
        # main.rs:1486-1671 restated op for op on both sides; only log10f may
        # differ by an ulp between the device and glibc (glibc's log10f is not
        # correctly rounded: 4% of floats differ from the rounded double log10).
        assert d.max() <= 2e-6, d.max()
        assert (got == ref).mean() > 0.9


def test_mel_empty_and_short(micro_ctx, oracle_micro):
    pcm = np.zeros(100, np.float32)  # < one hop: n_len = 0
    micro_ctx.pcm_to_mel_batch([pcm])
    assert micro_ctx.mel(0).shape == (80, 0)


def _check_encoder(ctx, om, pcm, n_ctx, mel_offset=0, pin=None):
    """Encoder output and cross K / V against the oracle (module docstring's
    bars); pin: additionally max |device - oracle| <= pin x floor (the
    round-5 verdict's "back under the floor", base and large-v3)."""
    enc_exact = _oracle_encode(om, pcm, n_ctx, mel_offset, exact=True)[0]
    enc_ref, ck_ref, cv_ref = _oracle_encode(om, pcm, n_ctx, mel_offset)
    floor = np.abs(enc_exact - enc_ref).max()
    floor_mean = np.abs(enc_exact - enc_ref).mean()
    ctx.set_audio_ctx(n_ctx)
    ctx.pcm_to_mel_batch([pcm])
    ctx.encode(1, mel_offset)
    enc = ctx.encoder_out(0)
    assert enc.shape == enc_ref.shape
    err = np.abs(enc - enc_ref)
    # reported per config (pytest -s / -rA): the literal north_star bound is 1e-3
    print(f"[encoder parity] n_state {enc.shape[1]} n_ctx {n_ctx}: max {err.max():.3e} mean {err.mean():.3e} "
          f"(noise floor max {floor:.3e} mean {floor_mean:.3e}; literal 1e-3 {'holds' if err.max() <= 1e-3 else 'exceeded'})")
    assert err.max() <= max(ENC_TOL, 1.25 * floor), (err.max(), floor)
    assert err.mean() <= max(3e-4, 1.25 * floor_mean), (err.mean(), floor_mean)
    if pin is not None:
        assert err.max() <= max(ENC_TOL, pin * floor), (err.max(), pin, floor)
    # the device result and the ggml-order oracle are two roundings of the
    # same exact (double-dot) result: the device must be as close to it as
    # ggml's own order is (scripts/enc_layer_err.py: ~1.0x at every layer of
    # small and small-q5_1, profiles/r03/enc_layers_*.log)
    err_x = np.abs(enc - enc_exact)
    print(f"[encoder parity] |device - exact| max {err_x.max():.3e} mean {err_x.mean():.3e}")
    assert err_x.max() <= max(ENC_TOL, 1.25 * floor), (err_x.max(), floor)
    assert err_x.mean() <= max(3e-4, 1.25 * floor_mean), (err_x.mean(), floor_mean)
    ck, cv = ctx.cross_kv(0)
    # cross K/V are f16 projections of the encoder output: same absolute
    # budget plus one f16 rounding of the stored value
    assert np.abs(f16(ck) - f16(ck_ref)).max() <= 2 * max(ENC_TOL, floor)
    assert np.abs(f16(cv) - f16(cv_ref)).max() <= 2 * max(ENC_TOL, floor)
    return enc_ref, ck_ref, cv_ref


def test_encoder_micro_short_ctx(micro_ctx, oracle_micro):
    _check_encoder(micro_ctx, oracle_micro, synth.synth_pcm_f32(2.0, 1234), 64)


def test_encoder_micro_ragged_ctx(micro_ctx, oracle_micro):
    # n_ctx not a multiple of 32 / 4 exercises every tile tail
    _check_encoder(micro_ctx, oracle_micro, synth.synth_pcm_f32(1.3, 11), 37)
    _check_encoder(micro_ctx, oracle_micro, synth.synth_pcm_f32(3.0, 12), 61, mel_offset=17)


def test_encoder_micro_full_ctx(micro_ctx, oracle_micro):
    _check_encoder(micro_ctx, oracle_micro, synth.synth_pcm_f32(30.0, 5), 1500)


def test_decoder_teacher_forced_logits(micro_ctx, oracle_micro):
    pcm = synth.synth_pcm_f32(2.0, 1234)
    enc_ref, ck_ref, cv_ref = _check_encoder(micro_ctx, oracle_micro, pcm, 64)
    rng = np.random.default_rng(0)
    toks = np.array(oracle_micro.prompt() + list(rng.integers(0, 50000, 10)), np.int32)
    ref = oracle_micro.decode_logits(ck_ref, cv_ref, toks, n_threads=threads())
    got = micro_ctx.decode_logits(toks, 0)
    err = np.abs(got - ref).max()
    assert err <= 2e-3, err
    top2 = np.sort(ref, axis=1)[:, -2:]
    decisive = (top2[:, 1] - top2[:, 0]) > 1e-3
    assert (got.argmax(1) == ref.argmax(1))[decisive].all()


def test_decoder_logits_full_text_ctx(micro_ctx, oracle_micro):
    """Maximum size: teacher-forced logits over the whole text context (448
    positions), so the self-attention runs every key-capacity bucket (64, 128,
    256, 512) and the KV cache fills to its last row; one token more is an
    error, not a silent overrun."""
    pcm = synth.synth_pcm_f32(2.0, 7)
    _, ck_ref, cv_ref = _check_encoder(micro_ctx, oracle_micro, pcm, 64)
    n_ctx = micro_ctx.hparams["n_text_ctx"]
    rng = np.random.default_rng(1)
    pr = oracle_micro.prompt()
    toks = np.array(pr + list(rng.integers(0, 50000, n_ctx - len(pr))), np.int32)
    ref = oracle_micro.decode_logits(ck_ref, cv_ref, toks, n_threads=threads())
    got = micro_ctx.decode_logits(toks, 0)
    err = np.abs(got - ref).max(axis=1)
    assert err.max() <= 2e-3, (err.max(), int(err.argmax()))
    top2 = np.sort(ref, axis=1)[:, -2:]
    decisive = (top2[:, 1] - top2[:, 0]) > 1e-3
    assert (got.argmax(1) == ref.argmax(1))[decisive].all()
    with pytest.raises(Exception):
        micro_ctx.decode_logits(np.concatenate([toks, toks[-1:]]), 0)


GREEDY_GAP = 1e-3  # oracle top-2 margins below this may flip under f32 reordering
# decoder logits: max |device - oracle| <= max(LOGIT_TOL, 1.25 x the logit
# noise floor), the floor being |oracle in ggml's order - oracle with exact
# (double) dots|, encoder included, on the same feed — the encoder bar's rule.
# Accepted departures from ggml's rounding points in the persistent decoder
# (they use part of the 1.25x headroom, so the large-v3 margin
# is pinned at 1.0x its floor in test_step_logits_one_row):
#  - self-attention: P V from the table values p, divided by the exact sum
#    afterwards (ggml rounds P16 = f16(p / sum) first);
#  - cross attention (flash-decoding): max, p and the exact sum per 128-key
#    sub-chunk, combined in f32 with e^(m - M) (ggml: one row max).
# The encoder attention keeps ggml's rounding points (P16 before P V).
LOGIT_TOL = 2e-3


def _exact_kv(om, pcm, n_ctx, mel_offset=0):
    """The oracle's cross K / V with exact (double) dot products."""
    return _oracle_encode(om, pcm, n_ctx, mel_offset, exact=True)[1:]


def _logits_ref(om, kv, kv_exact, feed):
    """Oracle teacher-forced logits of feed and the bar for the device's:
    (logits [len(feed)][V], bar, floor)."""
    feed = np.ascontiguousarray(feed, np.int32)
    lr = om.decode_logits(kv[0], kv[1], feed, n_threads=threads())
    pyoracle.set_dot_mode(True)
    try:
        lx = om.decode_logits(kv_exact[0], kv_exact[1], feed, n_threads=threads())
    finally:
        pyoracle.set_dot_mode(False)
    floor = float(np.abs(lr - lx).max())
    return lr, max(LOGIT_TOL, 1.25 * floor), floor


def _greedy_case(ctx, om, seeds, n_tok, n_ctx, secs, min_len):
    """Greedy ids against the oracle, all n_tok steps:
    - free running: identical up to the first difference, which may only
      fall on an oracle near-tie (top-2 margin < GREEDY_GAP: a different f32
      summation order may legitimately flip it);
    - teacher forced on the oracle's ids: the argmax (EOT suppressed, as in
      the greedy run) equals the oracle's id at every decisive step — at
      least min_len of them, or the next seed is tried.
    Returns (decisive steps compared, seed, the oracle's encoder outputs,
    pcm, oracle ids)."""
    tried = []
    for seed in seeds:
        pcm = synth.synth_pcm_f32(secs, seed)
        enc_ref, ck_ref, cv_ref = _check_encoder(ctx, om, pcm, n_ctx)
        ref, margins = om.decode_greedy(ck_ref, cv_ref, n_tok, suppress_eot=True, n_threads=threads())
        decisive = margins >= GREEDY_GAP
        tried.append((seed, int(decisive.sum())))
        if decisive.sum() < min_len:
            continue
        got = ctx.decode_greedy(n_tok, suppress_eot=True)[0]
        diff = np.nonzero(got != ref)[0]
        if diff.size:
            assert not decisive[diff[0]], (seed, int(diff[0]), float(margins[diff[0]]))
        prompt = list(om.prompt())
        feed = np.array(prompt + list(ref[:-1]), np.int32)
        lg = ctx.decode_logits(feed, 0)[len(prompt) - 1:]
        assert lg.shape[0] == n_tok
        # every teacher-forced position's logits, not only the argmax: a
        # cross K / V misalignment moves logits by ~0.1 with every argmax
        # unchanged (round-4 verdict)
        lr, bar, floor = _logits_ref(om, (ck_ref, cv_ref), _exact_kv(om, pcm, n_ctx), feed)
        err = float(np.abs(lg - lr[len(prompt) - 1:]).max())
        print(f"[greedy parity] seed {seed}: teacher-forced logits max |device - oracle| {err:.3e} over {n_tok} "
              f"positions (bar {bar:.3e}, floor {floor:.3e})")
        assert err <= bar, (err, bar)
        lg[:, om.special["eot"]] = -np.inf
        np.testing.assert_array_equal(lg.argmax(1)[decisive], ref[decisive])
        print(f"[greedy parity] seed {seed}: free-running ids identical for "
              f"{diff[0] if diff.size else n_tok} of {n_tok}; teacher-forced argmax identical at all "
              f"{int(decisive.sum())} decisive steps")
        return int(decisive.sum()), seed, (enc_ref, ck_ref, cv_ref), pcm, ref
    pytest.fail(f"no seed with >= {min_len} decisive greedy steps (seed, decisive): {tried}")


def test_greedy_tokens_micro(micro_ctx, oracle_micro):
    _greedy_case(micro_ctx, oracle_micro, range(99, 129), 24, 64, 2.0, min_len=18)


def test_batch_equals_single(micro_ctx):
    """A clip's encoder output is bitwise the same alone and in a batch; its
    greedy ids too (the multi-row decoder instance sums its GEMV dots on MFMA,
    the one-row instance on the VALU: each a fixed order, so the ids agree
    unless a step's top-2 logits are closer than the two orders' logit
    difference — measured at most 1.04e-3 at base, bounded by BATCH_GAP)."""
    clips = [synth.synth_pcm_f32(2.0, s) for s in (1, 2, 3)]
    micro_ctx.set_audio_ctx(64)
    micro_ctx.pcm_to_mel_batch(clips)
    micro_ctx.encode(1, 0)
    enc_b = [micro_ctx.encoder_out(i) for i in range(3)]
    tok_b = micro_ctx.decode_greedy(12, suppress_eot=True)
    for i, c in enumerate(clips):
        micro_ctx.pcm_to_mel_batch([c])
        micro_ctx.encode(1, 0)
        np.testing.assert_array_equal(micro_ctx.encoder_out(0), enc_b[i])
        _ids_agree_to_near_tie(micro_ctx, micro_ctx.decode_greedy(12, suppress_eot=True)[0], tok_b[i])


def test_staged_pipeline_matches_api(micro_ctx):
    clips = [synth.synth_pcm_f32(2.0, s) for s in (5, 6)]
    micro_ctx.set_audio_ctx(64)
    micro_ctx.stage(clips)
    micro_ctx.run_staged(n_decode=10)
    staged = micro_ctx.tokens()
    micro_ctx.pcm_to_mel_batch(clips)
    micro_ctx.encode(1, 0)
    api = micro_ctx.decode_greedy(10, suppress_eot=True)
    for i in range(2):
        np.testing.assert_array_equal(staged[i], api[i])
    t = micro_ctx.timings()
    assert t["decode_ms"] > 0 and t["encode_ms"] > 0


@pytest.mark.slow
@pytest.mark.parametrize("model", ["tiny.en", "base"])
def test_full_size_models(wmi, model_cache, model):
    path = synth.model_path(model, model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        if model == "base":  # C2's encoder under its floor (pinned)
            _check_encoder(ctx, om, synth.synth_pcm_f32(30.0, 1234), 1500, pin=1.0)
        _greedy_case(ctx, om, range(1234, 1240), 16, 1500, 30.0, min_len=12)
    finally:
        ctx.close()
        om.close()


# --- beam search (config C5; semantics restated in oracle/wmi_oracle.h) ------
BEAM_GAP = 2e-3  # selection margins below this may flip under f32 reordering


def _beam_case(ctx, om, seeds, K, n_tok, suppress_eot, n_ctx=64, secs=2.0, fail=False, min_tok=None,
               pcm_fn=synth.synth_pcm_f32, hyp_logits=False):
    """First seed whose oracle beam search has no near-tie selection (margin
    < BEAM_GAP) anywhere; the HIP path must then reproduce it exactly.  With
    min_tok, when every seed meets a near-tie, the seed whose first near-tie
    selection comes latest (step t >= min_tok) is compared over the t tokens
    before it — the searches agree step for step until then — provided that
    shorter search ends without a near-tie too."""
    best = None  # (t, seed, pcm)
    for seed in seeds:
        pcm = pcm_fn(secs, seed)
        _, ck, cv = _oracle_encode(om, pcm, n_ctx)
        ref, score, gap, sg = om.decode_beam(ck, cv, K, n_tok, suppress_eot=suppress_eot, n_threads=threads(),
                                             step_gaps=True)
        if gap < BEAM_GAP and min_tok:
            t = int(np.argmax(sg < BEAM_GAP)) if (sg < BEAM_GAP).any() else n_tok
            print(f"seed {seed}: first near-tie selection at step {t} (margins {np.round(sg, 5).tolist()})")
            while t >= min_tok and (best is None or t > best[0]):
                r2, s2, g2 = om.decode_beam(ck, cv, K, t, suppress_eot=suppress_eot, n_threads=threads())
                if g2 >= BEAM_GAP:
                    best = (t, pcm, r2, s2)
                    break
                t -= 1  # (a near-tie in the final ranking at this length)
            continue
        if gap >= BEAM_GAP:
            best = (n_tok, pcm, ref, score)
            break
    if best is not None:
        t, pcm, ref, score = best
        ctx.set_audio_ctx(n_ctx)
        ctx.pcm_to_mel_batch([pcm])
        ctx.encode(1, 0)
        got, got_score = ctx.decode_beam(K, t, suppress_eot=suppress_eot)[0]
        if hyp_logits:  # the winning hypothesis, teacher-forced through the one-row decoder
            feed = np.array(list(om.prompt()) + list(got[:-1]), np.int32)
            kv = _oracle_encode(om, pcm, n_ctx)[1:]
            lr, bar, floor = _logits_ref(om, kv, _exact_kv(om, pcm, n_ctx), feed)
            err = float(np.abs(ctx.decode_logits(feed, 0) - lr).max())
            print(f"[beam parity] K={K}: best hypothesis ({len(got)} tokens) teacher-forced logits max "
                  f"|device - oracle| {err:.3e} (bar {bar:.3e}, floor {floor:.3e})")
            assert err <= bar, (err, bar)
        return ref, score, got, got_score
    msg = f"no seed without a near-tie selection in {list(seeds)}"
    if fail:
        pytest.fail(msg)
    pytest.skip(msg)


@pytest.mark.parametrize("K", [1, 2, 3])
def test_beam_search_micro(micro_ctx, oracle_micro, K):
    ref, score, got, got_score = _beam_case(micro_ctx, oracle_micro, range(100, 130), K, 20, True)
    np.testing.assert_array_equal(got, ref)
    assert abs(got_score - score) < 1e-2


def test_beam_search_tiny_en_beam5(wmi, model_cache):
    """C5's beam width on a full-size model (the micro model's logits barely
    depend on the audio, so its 5-beam selections are all near-ties)."""
    path = synth.model_path("tiny.en", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        ref, score, got, got_score = _beam_case(ctx, om, range(1234, 1240), 5, 16, True, n_ctx=1500, secs=30.0)
        np.testing.assert_array_equal(got, ref)
        assert abs(got_score - score) < 1e-2
    finally:
        ctx.close()
        om.close()


@pytest.mark.parametrize("persist", ["0", "1"])
def test_beam_one_equals_greedy(wmi, micro_model, persist):
    """beam_size 1 == greedy, on the kernel chain (WMI_PERSIST=0) and on the
    default path (the persistent decoder: one beam-mode launch per step against
    the greedy launch of all steps)."""
    ctx = _ctx_with_env(wmi, micro_model, {"WMI_PERSIST": persist})
    try:
        ctx.set_audio_ctx(64)
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(2.0, 4)])
        ctx.encode(1, 0)
        g = ctx.decode_greedy(16, suppress_eot=True)[0]
        b, _ = ctx.decode_beam(1, 16, suppress_eot=True)[0]
        np.testing.assert_array_equal(b, g)
    finally:
        ctx.close()


def test_persistent_timeout_device_abort_and_fallback(wmi, micro_model):
    """WMI_FAULT_INJECT=1: the context's first persistent launch runs with its
    last workgroup missing (PersistArgs::stall_wg — a workgroup that never
    became resident).  Every other workgroup's poll of that workgroup's rows
    runs into the bounded spin, one of them raises the abort word and err bit
    3, and the whole grid drains (the device abort path, not a host-side
    mark).  The decode that failed is re-run on the kernel chain, which the
    context keeps from then on (one fallback counted, however many decodes
    follow).  Every decode kind that launches the persistent grid — greedy
    over two 8-row blocks, beam search, teacher-forced logits, a timestamp
    window — gives what a chain-only context gives."""
    import struct
    clips = [synth.synth_pcm_f32(2.0, 300 + i) for i in range(9)]  # two 8-row blocks
    feed = [50257, 50362, 100, 200, 300, 400]

    def run(env, kind):
        ctx = _ctx_with_env(wmi, micro_model, env, max_clips=9 if kind == "greedy" else 1)
        try:
            ctx.set_audio_ctx(64)
            ctx.pcm_to_mel_batch(clips if kind == "greedy" else clips[:1])
            ctx.encode(1, 0)
            if kind == "greedy":
                res = [list(t) for t in ctx.decode_greedy(10, suppress_eot=True)]
                res2 = [list(t) for t in ctx.decode_greedy(10, suppress_eot=True)]  # latched on the chain
                assert res2 == res
            elif kind == "beam":
                res = [(list(t), sc) for t, sc in ctx.decode_beam(2, 8, suppress_eot=True)]
            elif kind == "logits":
                res = ctx.decode_logits(feed)
            else:
                res = [(d["id"], d["tid"]) for d in ctx.decode_timestamps(feed[:1], 6)]
            return res, struct.unpack("<i", ctx.debug_read(11, 4))[0]
        finally:
            ctx.close()

    for kind in ("greedy", "beam", "logits", "timestamps"):
        got, fb = run({"WMI_FAULT_INJECT": "1"}, kind)
        want, fb0 = run({"WMI_PERSIST": "0"}, kind)
        assert fb == 1 and fb0 == 0, (kind, fb, fb0)
        if kind == "logits":
            np.testing.assert_array_equal(got, want)
        else:
            assert got == want, (kind, got, want)


@pytest.fixture(scope="module")
def eot_twin_model(model_cache):
    """micro with EOT's embedding row equal to the row greedy keeps choosing:
    EOT then ties the best candidate every step, so hypotheses finish and the
    finished-list / early-stop logic runs (exact ties, identical on both sides)."""
    import os
    path = os.path.join(model_cache, "ggml-synth-micro-eot-twin.bin")
    if not os.path.exists(path):
        def hook(name, arr):
            if name == "decoder.token_embedding.weight":
                arr = arr.copy()
                arr[50256] = arr[48938]
            return arr
        synth.write_ggml(path, "micro", tensor_hook=hook)
    return path


def test_beam_search_finishing(wmi, eot_twin_model):
    om = pyoracle.OracleModel(eot_twin_model)
    ctx = wmi.WhisperContext.new(eot_twin_model, 0, max_clips=1)
    try:
        for K in (2, 4):
            ref, score, got, got_score = _beam_case(ctx, om, range(200, 230), K, 30, False)
            assert ref[-1] == om.special["eot"]  # a finished hypothesis won
            np.testing.assert_array_equal(got, ref)
            assert abs(got_score - score) < 1e-2
    finally:
        ctx.close()
        om.close()


def test_base_batch_of_8_equals_single(wmi, model_cache):
    """C4's per-GPU shard: 8 x 30 s clips through the batched encoder (M =
    12000 rows per GEMM) and the 8-row persistent decoder give the single-clip
    results (which the full-size test pins to the oracle): encoder output
    bitwise; greedy ids equal up to a near-tie of the one-row decoder
    (BATCH_GAP).  The one-row instance sums its GEMV dots on the VALU, the
    multi-row one on MFMA: where a clip's ids agree, the last step's logits of
    the two are compared and their largest difference printed and bounded."""
    ctx = _ctx_with_env(wmi, synth.model_path("base", model_cache), {"WMI_PERSIST_LOGITS": "1"}, max_clips=8)
    try:
        V = ctx.hparams["n_vocab"]
        clips = [synth.synth_pcm_f32(30.0, 1234 + i) for i in range(8)]
        ctx.pcm_to_mel_batch(clips)
        ctx.encode(1, 0)
        enc_b = [ctx.encoder_out(i) for i in range(8)]
        tok_b = ctx.decode_greedy(12, suppress_eot=True)
        lg_b = np.frombuffer(ctx.debug_read(2, 8 * V * 4), np.float32).reshape(8, V).copy()
        worst = 0.0
        for i in range(8):
            ctx.pcm_to_mel_batch([clips[i]])
            ctx.encode(1, 0)
            np.testing.assert_array_equal(ctx.encoder_out(0), enc_b[i])
            single = ctx.decode_greedy(12, suppress_eot=True)[0]
            if (single == tok_b[i]).all():
                lg1 = np.frombuffer(ctx.debug_read(2, V * 4), np.float32)
                worst = max(worst, float(np.abs(lg1 - lg_b[i]).max()))
            else:
                _ids_agree_to_near_tie(ctx, single, tok_b[i])
        print(f"[batch scope] base: max |logit(B=1) - logit(B=8)| at the last step = {worst:.3g}")
        assert worst <= BATCH_GAP
    finally:
        ctx.close()


@pytest.mark.slow
def test_large_v3(wmi, model_cache):
    """C5's model: 128 mels, vocab 51866 (multilingual specials shifted by one
    more id), n_state 1280 / 20 heads / 32 + 32 layers; encoder at the noise
    floor (pinned: the two-key-part attention, attn_enc_kq), greedy ids
    (>= 9 of 12 compared) and teacher-forced logits.  (Its 5-beam search meets
    a near-tie selection within 5-12 steps on every seed, so C5's beam launch
    is held to the oracle step by step on large-v3-xsharp instead:
    test_beam_step_logits_large_v3_xsharp.)"""
    path = synth.model_path("large-v3", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        assert ctx.hparams["n_mels"] == 128 and ctx.hparams["n_vocab"] == 51866
        _check_encoder(ctx, om, synth.synth_pcm_f32(30.0, 1234), 1500, pin=1.0)
        _greedy_case(ctx, om, range(1234, 1237), 12, 1500, 30.0, min_len=9)
    finally:
        ctx.close()
        om.close()


# --- long decode horizons (round-4 verdict item 4) ----------------------------
# The plain random models meet a top-2 near-tie within 7-12 steps, which caps
# how far their ids can be compared.  The "-sharp" variants (synth.sharp_hook:
# token embedding x 4, positional embedding x 100) keep every decision far
# above f32 reordering noise, so the ids are compared over the whole horizon.
@pytest.mark.slow
def test_long_horizon_greedy_base_sharp(wmi, model_cache):
    """base-sharp, 96 greedy tokens: one clip (the one-row instance) and 8
    clips (C4's shard, the 8-row instance) against the oracle, id for id over
    at least 64 decisive steps; teacher-forced argmax identical at every
    decisive step."""
    path = synth.model_path("base-sharp", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=8)
    n_tok = 96
    try:
        n_dec, seed, _, _, ref = _greedy_case(ctx, om, range(1234, 1240), n_tok, 1500, 30.0, min_len=64)
        seeds = [1234 + i for i in range(8)]
        clips = [synth.synth_pcm_f32(30.0, sd) for sd in seeds]
        ctx.pcm_to_mel_batch(clips)
        ctx.encode(1, 0)
        got8 = ctx.decode_greedy(n_tok, suppress_eot=True)
        same = 0
        for i, pcm in enumerate(clips):
            _, ck, cv = _oracle_encode(om, pcm, 1500)
            r, m = om.decode_greedy(ck, cv, n_tok, suppress_eot=True, n_threads=threads())
            diff = np.nonzero(got8[i] != r)[0]
            if diff.size:
                assert m[diff[0]] < GREEDY_GAP, (i, int(diff[0]), float(m[diff[0]]))
            same += int(diff[0]) if diff.size else n_tok
            assert (m >= GREEDY_GAP).sum() >= 64
        print(f"[long horizon] base-sharp: 1 clip {n_dec} decisive of {n_tok}; 8 clips: {same} of {8 * n_tok} "
              f"ids identical to the oracle before any near-tie")
        assert same >= 8 * 64
    finally:
        ctx.close()
        om.close()


@pytest.mark.slow
def test_long_horizon_beam_large_v3_sharp(wmi, model_cache):
    """large-v3-sharp, C5's search (5 beams, EOT suppressed) over 40 tokens:
    the ids equal the oracle's, compared over at least 32 tokens."""
    path = synth.model_path("large-v3-sharp", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        ref, score, got, got_score = _beam_case(ctx, om, range(1234, 1237), 5, 40, True, n_ctx=1500, secs=30.0,
                                                fail=True, min_tok=32, hyp_logits=True)
        print(f"[long horizon] large-v3-sharp 5-beam ids compared over {len(ref)} tokens")
        assert len(ref) >= 32
        np.testing.assert_array_equal(got, ref)
        assert abs(got_score - score) < 2e-2
    finally:
        ctx.close()
        om.close()


def test_multirow_instances_bitwise_independent_of_B(wmi, model_cache):
    """The multi-row persistent instance (2 <= B <= 8 rows) gives every row the
    same arithmetic whatever B is (MSet: one fixed MFMA / wave-order chain per
    (weight row, decoder row); one partial per 128 keys in the cross softmax):
    clips decoded as B = 2, 3 and 8 give bitwise the same ids and last-step
    logits.  (B = 1 runs the VALU GEMVs: see test_batch_equals_single.)"""
    path = synth.model_path("base", model_cache)
    clips = [synth.synth_pcm_f32(30.0, 1234 + i) for i in range(8)]
    V = None
    res = {}
    for nb in (8, 3, 2):
        ctx = _ctx_with_env(wmi, path, {"WMI_PERSIST_LOGITS": "1"}, max_clips=nb)
        try:
            V = ctx.hparams["n_vocab"]
            ctx.pcm_to_mel_batch(clips[:nb])
            ctx.encode(1, 0)
            toks = ctx.decode_greedy(24, suppress_eot=True)
            lg = np.frombuffer(ctx.debug_read(2, nb * V * 4), np.float32).reshape(nb, V).copy()
            res[nb] = (toks, lg)
        finally:
            ctx.close()
    for nb in (3, 2):
        for i in range(nb):
            np.testing.assert_array_equal(res[nb][0][i], res[8][0][i])
            np.testing.assert_array_equal(res[nb][1][i], res[8][1][i])


def test_encoder_gemm_paths_bitwise(wmi, model_cache):
    """The 8-clip encoder's GEMMs run on the LDS-DMA kernel (k_gemm_g) and
    the one-clip ones on its LDS-DMA ring form (k_gemm_p), with epilogues
    staged through LDS; WMI_GEMM_G=0 / WMI_GEMM_P=0 select the
    register-staged kernel (k_gemm), WMI_GEMM_EPI=0 the per-lane epilogue
    stores, WMI_GELU_CALC=0 the GELU table for every input (by default the
    epilogues compute the table's values above the context's scanned
    threshold).  All give
    bitwise the same encoder output and cross K / V (one MFMA order; one
    f32 -> f16 rounding sequence, f16_rt), at 8 clips and one clip."""
    path = synth.model_path("base", model_cache)
    clips = [synth.synth_pcm_f32(30.0, 1400 + i) for i in range(8)]
    for nc in (8, 1):
        ref = None
        for env in ({}, {"WMI_GEMM_EPI": "0"}, {"WMI_GEMM_G": "0"}, {"WMI_GEMM_G": "0", "WMI_GEMM_EPI": "0"},
                    {"WMI_GEMM_P": "0"}, {"WMI_GEMM_P": "0", "WMI_GEMM_EPI": "0"}, {"WMI_GELU_CALC": "0"},
                    {"WMI_GELU_CALC": "0", "WMI_GEMM_EPI": "0"}):
            ctx = _ctx_with_env(wmi, path, env, max_clips=nc)
            try:
                # the GELU epilogues' threshold: computed at or above it, the
                # table below (+inf with WMI_GELU_CALC=0); the device's tanhf
                # rounds to the table's f16 for every input (the scan: -inf)
                gmin = float(np.frombuffer(ctx.debug_read(18, 4), np.float32)[0])
                if env.get("WMI_GELU_CALC") == "0":
                    assert gmin == np.inf
                else:
                    assert gmin < 0.0, gmin
                ctx.pcm_to_mel_batch(clips[:nc])
                ctx.encode(1, 0)
                got = [(ctx.encoder_out(i), *ctx.cross_kv(i)) for i in range(nc)]
            finally:
                ctx.close()
            if ref is None:
                ref = got
                continue
            for a, b in zip(ref, got):
                for x, y in zip(a, b):
                    np.testing.assert_array_equal(x, y)


def test_split_grid_equals_full_grid(wmi, model_cache):
    """A block of 8 clips decodes as two concurrent half-grid launches (rows
    0-3 and 4-7 on 128 workgroups each, two streams, separate exchange blocks,
    cache rows and argmax carries): bitwise the ids and every step's logits
    (WMI_LOGITS_ALL: all 41 positions of every row) of the one full-grid
    launch (WMI_SPLIT_ROWS=0) — the row partition of the multi-row phases
    changes which workgroup computes a dot, not its order."""
    path = synth.model_path("base", model_cache)
    clips = [synth.synth_pcm_f32(30.0, 1300 + i) for i in range(8)]
    res = []
    for env in ({"WMI_SPLIT_ROWS": "8"}, {"WMI_SPLIT_ROWS": "0"}):
        ctx = _ctx_with_env(wmi, path, dict(env, WMI_LOGITS_ALL="1"), max_clips=8)
        try:
            ctx.pcm_to_mel_batch(clips)
            ctx.encode(1, 0)
            toks = ctx.decode_greedy(40, suppress_eot=True)
            res.append((toks, ctx.step_logits(len(_prompt(ctx)) + 40 - 1)))
        finally:
            ctx.close()
    for i in range(8):
        np.testing.assert_array_equal(res[0][0][i], res[1][0][i])
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_gelu_calc_equals_table_decode(wmi, model_cache):
    """The persistent decoder's phase H computes GELU where the context's scan
    allows (gelu_bits) instead of gathering ggml's table: bitwise the ids and
    every step's logits of the table-only context (WMI_GELU_CALC=0), on the
    one-row instance and the 8-row split grid, encoder included."""
    path = synth.model_path("base", model_cache)
    for nc in (1, 8):
        clips = [synth.synth_pcm_f32(30.0, 1500 + i) for i in range(nc)]
        res = []
        for env in ({}, {"WMI_GELU_CALC": "0"}):
            ctx = _ctx_with_env(wmi, path, dict(env, WMI_LOGITS_ALL="1"), max_clips=nc)
            try:
                ctx.pcm_to_mel_batch(clips)
                ctx.encode(1, 0)
                toks = ctx.decode_greedy(40, suppress_eot=True)
                res.append((toks, ctx.step_logits(len(_prompt(ctx)) + 40 - 1)))
            finally:
                ctx.close()
        for i in range(nc):
            np.testing.assert_array_equal(res[0][0][i], res[1][0][i])
        np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.slow
def test_beam_shared_cross_equals_per_row(wmi, model_cache):
    """C5's beam rows read their clip's cross K / V through one task per (head,
    key chunk) (PersistArgs::xshare): bitwise the tokens and scores of the
    per-row tasks (WMI_XSHARE=0), whose arithmetic it repeats row by row."""
    path = synth.model_path("large-v3", model_cache)
    pcm = [synth.synth_pcm_f32(30.0, 1236)]
    out = []
    for env in ({}, {"WMI_XSHARE": "0"}):
        ctx = _ctx_with_env(wmi, path, env)
        try:
            ctx.pcm_to_mel_batch(pcm)
            ctx.encode(1, 0)
            out.append(ctx.decode_beam(5, 16, suppress_eot=True)[0])
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


# --- ggml quantised weights (config C3; semantics in tests/test_quant.py) ----
@pytest.mark.parametrize("qtype", ["q4_0", "q4_1", "q5_0", "q5_1", "q8_0"])
def test_quantised_micro(wmi, model_cache, qtype):
    import os
    path = os.path.join(model_cache, f"ggml-synth-micro-{qtype}.bin")
    if not os.path.exists(path):
        synth.write_ggml(path, "micro", quant=qtype)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        _, ck_ref, cv_ref = _check_encoder(ctx, om, synth.synth_pcm_f32(2.0, 1234), 64)
        toks = np.array(om.prompt() + [1000, 2000, 3000], np.int32)
        ref = om.decode_logits(ck_ref, cv_ref, toks, n_threads=threads())
        assert np.abs(ctx.decode_logits(toks, 0) - ref).max() <= 2e-3
    finally:
        ctx.close()
        om.close()


def test_small_q5_1(wmi, model_cache):
    """C3: whisper small with q5_1 weights.  Every decoder path is held to
    the oracle: the default (persistent) decoder, the kernel chain streaming
    the q5_1 blocks (dequantised in registers to exactly the loader's f16
    weights), and the chain on the dequantised f16 copies (WMI_NO_Q5=1)."""
    path = synth.model_path("small-q5_1", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    chain5 = _ctx_with_env(wmi, path, {"WMI_PERSIST": "0"})
    chain16 = _ctx_with_env(wmi, path, {"WMI_PERSIST": "0", "WMI_NO_Q5": "1"})
    try:
        _, seed, (_, ck_ref, cv_ref), pcm, ref = _greedy_case(ctx, om, range(1234, 1238), 16, 1500, 30.0,
                                                              min_len=12)
        for c in (chain5, chain16):
            _greedy_case(c, om, [seed], 16, 1500, 30.0, min_len=12)
        toks = np.array(om.prompt() + list(ref[:6]), np.int32)
        lref = om.decode_logits(ck_ref, cv_ref, toks, n_threads=threads())
        errs = [np.abs(c.decode_logits(toks, 0) - lref).max() for c in (ctx, chain5, chain16)]
        assert max(errs) <= 5e-3, errs
    finally:
        chain16.close()
        chain5.close()
        ctx.close()
        om.close()


@pytest.mark.parametrize("model,n_clips", [("micro-q5_1", 1), ("micro-q5_1", 3), ("small-q5_1", 1),
                                           ("small-q5_1", 2)])
def test_persistent_q5_equals_f16(wmi, model_cache, model, n_clips):
    """The persistent decoder's q5_1 instances (phases A, C, G2, H, I stream
    the q5_1 blocks and dequantise them in registers) give bitwise the ids and
    step logits of its f16 instances on the loader's dequantised copies
    (WMI_NO_Q5=1): both multiply the same f16 weights in the same order."""
    import os
    if model == "micro-q5_1":
        path = os.path.join(model_cache, "ggml-synth-micro-q5_1.bin")
        if not os.path.exists(path):
            synth.write_ggml(path, "micro", quant="q5_1")
        secs, n_ctx = 2.0, 64
    else:
        path, secs, n_ctx = synth.model_path(model, model_cache), 30.0, 1500
    clips = [synth.synth_pcm_f32(secs, 70 + i) for i in range(n_clips)]
    ctxs = [_ctx_with_env(wmi, path, env, max_clips=n_clips)
            for env in ({"WMI_PERSIST_LOGITS": "1", "WMI_PERSIST_Q5": "1"}, {"WMI_PERSIST_LOGITS": "1", "WMI_NO_Q5": "1"})]
    try:
        out = []
        for ctx in ctxs:
            ctx.set_audio_ctx(n_ctx)
            ctx.pcm_to_mel_batch(clips)
            ctx.encode(1, 0)
            toks = ctx.decode_greedy(24, suppress_eot=True)
            V = ctx.hparams["n_vocab"]  # last step's logits, rows [n_clips][V] (WMI_PERSIST_LOGITS)
            out.append((toks, np.frombuffer(ctx.debug_read(2, n_clips * V * 4), np.float32).copy()))
        for i in range(n_clips):
            np.testing.assert_array_equal(out[0][0][i], out[1][0][i])
        np.testing.assert_array_equal(out[0][1], out[1][1])
    finally:
        for ctx in ctxs:
            ctx.close()


@pytest.mark.parametrize("model,n_clips,n_ctx", [("micro", 1, 64), ("micro", 3, 64), ("micro", 2, 1500),
                                                 ("tiny.en", 1, 1500), ("base", 2, 1500)])
def test_persistent_matches_chain(wmi, model_cache, model, n_clips, n_ctx):
    """The persistent decoder (every greedy step of a run in one launch,
    phases handed off through sc1 granules) against the kernel chain with the
    unfused output projection (WMI_NO_FUSE=1), which computes each op in the
    same f32 order except the self-attention/cross-attention partial sums:
    teacher-forced logits agree within 2e-3 at every position, and the greedy
    ids of a 40-step run are identical up to the first step whose top-2 margin
    (in the chain's own teacher-forced logits) is below 2e-3 — a near-tie a
    last-bit difference may legitimately flip (base seed 41: one at step 10,
    margin 4.9e-4 in the oracle)."""
    path = synth.model_path(model, model_cache)
    clips = [synth.synth_pcm_f32(30.0 if n_ctx == 1500 else 2.0, 40 + i) for i in range(n_clips)]
    ctxs = [_ctx_with_env(wmi, path, env, max_clips=n_clips)
            for env in ({"WMI_PERSIST": "1"}, {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})]
    try:
        out = []
        for ctx in ctxs:
            ctx.set_audio_ctx(n_ctx)
            ctx.pcm_to_mel_batch(clips)
            ctx.encode(1, 0)
            out.append(ctx.decode_greedy(40, suppress_eot=True))
        for i in range(n_clips):
            tp, tc = out[0][i], out[1][i]
            feed = np.concatenate([_prompt(ctxs[1]), tc[:-1]]).astype(np.int32)
            lp, lc = (ctx.decode_logits(feed, i) for ctx in ctxs)
            assert np.abs(lp - lc).max() <= 2e-3, np.abs(lp - lc).max()
            np_ = len(feed) - len(tc) + 1
            top2 = np.sort(lc[np_ - 1:], axis=1)[:, -2:]
            margin = top2[:, 1] - top2[:, 0]
            diff = np.nonzero(tp != tc)[0]
            if diff.size:
                assert margin[diff[0]] < 2e-3, (diff[0], margin[diff[0]])
            assert (tp[:diff[0] if diff.size else len(tp)] == tc[:diff[0] if diff.size else len(tc)]).all()
    finally:
        for ctx in ctxs:
            ctx.close()


# one-row (VALU GEMV) vs multi-row (MFMA GEMV) logits differ by up to ~1e-3
# (1.04e-3 measured at base over 8 clips x 51865 logits; an f32 reordering
# that flips one f16 rounding point inside a layer moves the logits by about
# that much): ids may part only where the top-2 margin is below 2x that.
# test_base_batch_of_8_equals_single measures and bounds it.
BATCH_GAP = 2e-3


def _ids_agree_to_near_tie(ctx, single, batched, gap=BATCH_GAP):
    """Greedy ids of clip 0 decoded alone vs in a batch: identical up to the
    first difference, which may only fall on a step whose top-2 margin (in
    the one-row decoder's teacher-forced logits of the single run) is < gap,
    the bound on the two instances' logit difference; nothing after the first
    difference is compared (the histories differ from there)."""
    diff = np.nonzero(np.asarray(single) != np.asarray(batched))[0]
    if not diff.size:
        return
    d = int(diff[0])
    feed = np.concatenate([_prompt(ctx), np.asarray(single[:d], np.int32)]).astype(np.int32)
    lg = ctx.decode_logits(feed, 0)[-1].copy()
    lg[ctx.special["eot"]] = -np.inf  # (the greedy runs suppress EOT)
    top2 = np.sort(lg)[-2:]
    assert top2[1] - top2[0] < gap, (d, float(top2[1] - top2[0]))


def _prompt(ctx):
    sp = ctx.special  # prompt_tokens (wmi_api.cpp): [SOT (, <|en|>, transcribe), NOT]
    if sp["multilingual"]:
        return np.array([sp["sot"], sp["sot"] + 1, sp["transcribe"], sp["not"]], np.int32)
    return np.array([sp["sot"], sp["not"]], np.int32)


def _ctx_with_env(wmi, path, env, max_clips=1):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return wmi.WhisperContext.new(path, 0, max_clips=max_clips)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("K", [2, 3])
def test_beam_rows_cross_attention(wmi, micro_model, oracle_micro, K):
    """Two-kernel cross-attention (WMI_NO_COOP=1) with beam rows sharing one
    workgroup per (chunk, head) (k_dec_xattn_rows, forced with WMI_XATTN_ROWS=2): the oracle's beams, and
    tokens and scores bit-identical to one workgroup per row
    (WMI_XATTN_ROWS=0).  The fused output projection's residual update runs
    inside the row loop at these sizes."""
    rows = _ctx_with_env(wmi, micro_model, {"WMI_PERSIST": "0", "WMI_NO_COOP": "1", "WMI_XATTN_ROWS": "2"})
    try:
        ref, score, got, got_score = _beam_case(rows, oracle_micro, range(100, 130), K, 20, True)
        np.testing.assert_array_equal(got, ref)
        assert abs(got_score - score) < 1e-2
    finally:
        rows.close()
    per = _ctx_with_env(wmi, micro_model, {"WMI_PERSIST": "0", "WMI_NO_COOP": "1", "WMI_XATTN_ROWS": "0"})
    try:
        ref2, score2, got2, got_score2 = _beam_case(per, oracle_micro, range(100, 130), K, 20, True)
        np.testing.assert_array_equal(got2, got)
        assert got_score2 == got_score
    finally:
        per.close()


def test_beam_rows_tiny_en_beam5_identical(wmi, model_cache):
    """C5's width at full audio context: k_dec_xattn_rows (5 rows, 12 chunks)
    gives the same beams and scores, bit for bit, as per-row workgroups."""
    path = synth.model_path("tiny.en", model_cache)
    pcm = synth.synth_pcm_f32(30.0, 1234)
    out = []
    for rows in ("2", "0", "1"):
        ctx = _ctx_with_env(wmi, path, {"WMI_PERSIST": "0", "WMI_NO_COOP": "1", "WMI_XATTN_ROWS": rows})
        try:
            ctx.set_audio_ctx(1500)
            ctx.pcm_to_mel_batch([pcm])
            ctx.encode(1, 0)
            out.append(ctx.decode_beam(5, 24, suppress_eot=True)[0])
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_persistent_beam_matches_chain(wmi, model_cache):
    """Beam search on the persistent decoder (one launch per step with the
    beam slots as rows, the history table for self-attention keys, the beam
    kernels between launches) against the kernel chain's beam search: the
    same 5-beam hypothesis at C5's width over the full audio context."""
    path = synth.model_path("tiny.en", model_cache)
    pcm = synth.synth_pcm_f32(30.0, 1234)
    out = []
    for env in ({"WMI_PERSIST": "1"}, {"WMI_PERSIST": "0"}):
        ctx = _ctx_with_env(wmi, path, env)
        try:
            ctx.set_audio_ctx(1500)
            ctx.pcm_to_mel_batch([pcm])
            ctx.encode(1, 0)
            out.append(ctx.decode_beam(5, 24, suppress_eot=True)[0])
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert abs(out[0][1] - out[1][1]) < 1e-2, (out[0][1], out[1][1])  # the oracle tests' bound


def test_reference_checksums(wmi, micro_model, oracle_micro):
    """The reference's stage sums from the HIP path (WMI_CHECKSUMS=1) against
    the oracle's: model-only and host sums exactly, the two mel sums within
    the mel's own tolerance (<= 2e-6 a value, summed sequentially)."""
    ctx = _ctx_with_env(wmi, micro_model, {"WMI_CHECKSUMS": "1"})
    try:
        pcm = synth.synth_pcm_f32(3.0, 77)
        ctx.set_audio_ctx(64)
        ctx.pcm_to_mel_batch([pcm])
        ctx.encode(1, 17)
        got = ctx.checksums()
        ref = oracle_micro.checksums(pcm, mel_offset=17, n_ctx=64)
        print(f"[checksums] hip {got} oracle {ref}")
        for k in ("hann", "samples", "filters"):
            assert got[k] == ref[k], (k, got[k], ref[k])
        n = 80 * 300
        for k in ("mel_raw", "mel_window"):
            assert abs(got[k] - ref[k]) <= 2e-6 * n + 1e-5 * abs(ref[k]), (k, got[k], ref[k])
    finally:
        ctx.close()


@pytest.mark.parametrize("model,n_ctx,secs", [("micro-f32", 64, 2.0), ("tiny.en-f32", 1500, 30.0)])
def test_f32_model(wmi, model_cache, model, n_ctx, secs):
    """ftype-0 (f32) files (main.rs:817-821, 1423-1427): f32 MFMA GEMMs for the
    conv stem / encoder / cross K/V and f32 decoder GEMVs, neither operand
    rounded to f16 (wmi_f32.hip), held to the oracle's f32 path: the encoder
    bar, greedy ids over every decisive step, teacher-forced logits, beam K=2."""
    path = synth.model_path(model, model_cache)
    om = pyoracle.OracleModel(path)
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        assert om.hp["f16"] == 0
        _, seed, (_, ck_ref, cv_ref), pcm, ref = _greedy_case(ctx, om, range(99, 129), 16, n_ctx, secs, min_len=12)
        toks = np.array(om.prompt() + list(ref[:8]), np.int32)
        lref = om.decode_logits(ck_ref, cv_ref, toks, n_threads=threads())
        err = np.abs(ctx.decode_logits(toks, 0) - lref).max()
        print(f"[f32 parity] {model}: teacher-forced logits max err {err:.3e}")
        assert err <= 2e-3, err
        if model == "micro-f32":
            bref, score, got, got_score = _beam_case(ctx, om, range(100, 130), 2, 12, True)
            np.testing.assert_array_equal(got, bref)
            assert abs(got_score - score) < 1e-2
    finally:
        ctx.close()
        om.close()


@pytest.mark.parametrize("nw", ["0", "1", "2", "4"])
def test_enc_attn_nw_parity_and_batch_invariance(wmi, model_cache, nw):
    """k_attn_enc4 with 1, 2 and 4 query blocks per workgroup (WMI_ENC_ATTN_NW;
    0: the default, 2 at one clip of base and 4 at eight): the encoder bar
    against the oracle at base's full 1500 frames, and a clip's result bitwise
    independent of the batch (8 clips vs 1) — across the default's switch too."""
    path = synth.model_path("base", model_cache)
    om = pyoracle.OracleModel(path)
    ctx = _ctx_with_env(wmi, path, {"WMI_ENC_ATTN_NW": nw}, max_clips=8)
    try:
        pcm = synth.synth_pcm_f32(30.0, 1234)
        _check_encoder(ctx, om, pcm, 1500)
        single = ctx.encoder_out(0)
        clips = [synth.synth_pcm_f32(30.0, 1234 + i) for i in range(8)]
        ctx.pcm_to_mel_batch(clips)
        ctx.encode(1, 0)
        np.testing.assert_array_equal(ctx.encoder_out(0), single)
    finally:
        ctx.close()
        om.close()


# --- every step's logits of the persistent greedy launches (round-4 verdict
# item 1): the device's own free-running decode, its logits at every position
# (WMI_LOGITS_ALL), against the oracle teacher-forced on the device's ids -----
def _step_logits_case(wmi, om, path, clips, n_tok, env=None, tag="", floor_clips=None, pin=None, n_ctx=1500):
    """Greedy-decode the clips in one call (8 clips: the split 8-row grid
    where the model has one; 2-8 clips: one multi-row launch; 1 clip: the
    one-row instance) with every position's logits kept.  Per clip: logits
    at every step within the bar of _logits_ref; the device's ids are the
    argmax of its own logits (EOT suppressed); the oracle's argmax on the
    device's history equals the device's id at every decisive step (oracle
    top-2 margin >= GREEDY_GAP) — so the oracle's own free-running decode
    gives the device's ids up to its first near-tie (both histories are equal
    until then).  floor_clips: measure the exact-dot floor on the first
    floor_clips clips only and hold the others to the largest of those bars
    (a large-v3 exact encode is ~30 s of host time).  pin: additionally
    max |device - oracle| <= max(LOGIT_TOL, pin x floor) (the margin the
    accepted softmax departures leave, LOGIT_TOL's comment).  Returns the
    device ids and the per-clip decisive step counts."""
    ctx = _ctx_with_env(wmi, path, dict(env or {}, WMI_LOGITS_ALL="1"), max_clips=len(clips))
    try:
        ctx.set_audio_ctx(n_ctx)
        ctx.pcm_to_mel_batch(clips)
        ctx.encode(1, 0)
        got = ctx.decode_greedy(n_tok, suppress_eot=True)
        prompt = list(om.prompt())
        np_ = len(prompt)
        lg_all = ctx.step_logits(np_ + n_tok - 1)
    finally:
        ctx.close()
    eot = om.special["eot"]
    worst, worst_bar, n_dec, bars = 0.0, 0.0, [], []
    n_floor = len(clips) if floor_clips is None else floor_clips
    for i, pcm in enumerate(clips):
        g = np.asarray(got[i])
        kv = _oracle_encode(om, pcm, n_ctx)[1:]
        feed = np.array(prompt + list(g[:-1]), np.int32)
        if i < n_floor:
            lr, bar, floor = _logits_ref(om, kv, _exact_kv(om, pcm, n_ctx), feed)
            bars.append((bar, floor))
        else:
            lr = om.decode_logits(kv[0], kv[1], feed, n_threads=threads())
            bar, floor = max(bars)
        lr = lr[np_ - 1:]
        lg = lg_all[np_ - 1:, i, :]
        err = float(np.abs(lg - lr).max())
        worst, worst_bar = max(worst, err), max(worst_bar, bar)
        assert err <= bar, (tag, i, err, bar, floor)
        if pin is not None:
            assert err <= max(LOGIT_TOL, pin * floor), (tag, i, err, pin, floor)
        lg[:, eot] = -np.inf
        np.testing.assert_array_equal(lg.argmax(1), g)  # the ids are the logits' argmax
        lr[:, eot] = -np.inf
        top2 = np.sort(lr, axis=1)[:, -2:]
        decisive = (top2[:, 1] - top2[:, 0]) >= GREEDY_GAP
        ora = lr.argmax(1)
        np.testing.assert_array_equal(ora[decisive], g[decisive])
        diff = np.nonzero(ora != g)[0]
        n_dec.append(int(decisive.sum()))
        print(f"[step logits] {tag} clip {i}: {n_tok} steps, max |device - oracle| {err:.3e} (bar {bar:.3e}, "
              f"floor {floor:.3e}{'' if i < n_floor else ' of clip 0'}); {n_dec[-1]} decisive; ids = the oracle's "
              f"argmax on the same history for {int(diff[0]) if diff.size else n_tok} steps")
    print(f"[step logits] {tag}: worst {worst:.3e} (largest bar {worst_bar:.3e}); "
          f"{len({tuple(x) for x in got})} distinct id sequences over {len(clips)} clips")
    return got, n_dec


@pytest.mark.slow
@pytest.mark.parametrize("model,n_tok,env", [
    ("base", 128, {}),                         # C2's instance on the bench's own clip: <512,1>
    ("small", 48, {}),                         # <768,1> with register-resident vocabulary rows
    ("small-q5_1", 48, {}),                    # C3: <768,1,Q5>
    ("large-v3", 24, {}),                      # <1280,1>
])
def test_step_logits_one_row(wmi, model_cache, model, n_tok, env):
    path = synth.model_path(model, model_cache)
    om = pyoracle.OracleModel(path)
    try:
        _step_logits_case(wmi, om, path, [synth.synth_pcm_f32(30.0, 1234)], n_tok, env, tag=f"{model} x1",
                          pin=1.0 if model == "large-v3" else None)
    finally:
        om.close()


def test_xsharp_ids_follow_the_audio_and_match(wmi, model_cache):
    """base-xsharp (synth.xsharp_hook: the audio drives the ids) on 8 tone
    clips (synth.synth_pcm_tones), 96 greedy tokens: the 8-row split grid in
    one call and every clip again alone on the one-row instance, each step's
    logits within the bar and the ids = the oracle's; at least 6 distinct id
    sequences (a row / clip routing or cross K / V indexing bug changes a
    compared id), at least 64 decisive steps per clip."""
    path = synth.model_path("base-xsharp", model_cache)
    om = pyoracle.OracleModel(path)
    n_tok = 96
    try:
        clips = [synth.synth_pcm_tones(30.0, 1234 + i) for i in range(8)]
        got8, dec8 = _step_logits_case(wmi, om, path, clips, n_tok, tag="base-xsharp x8 (split 8-row grid)")
        assert len({tuple(x) for x in got8}) >= 6
        assert min(dec8) >= 64, dec8
        for i, pcm in enumerate(clips):
            got1, _ = _step_logits_case(wmi, om, path, [pcm], n_tok, tag=f"base-xsharp clip {i} one-row")
            _ids_agree_to_near_tie_oracle(om, pcm, got1[0], got8[i])
    finally:
        om.close()


def _ids_agree_to_near_tie_oracle(om, pcm, a, b, gap=BATCH_GAP):
    """Two device decodes of one clip (one-row vs 8-row instance): identical
    up to a first difference on a step whose oracle top-2 margin is < gap."""
    diff = np.nonzero(np.asarray(a) != np.asarray(b))[0]
    if not diff.size:
        return
    d = int(diff[0])
    kv = _oracle_encode(om, pcm, 1500)[1:]
    lg = om.decode_logits(kv[0], kv[1], np.array(list(om.prompt()) + list(a[:d]), np.int32), n_threads=threads())[-1]
    lg[om.special["eot"]] = -np.inf
    top2 = np.sort(lg)[-2:]
    assert top2[1] - top2[0] < gap, (d, float(top2[1] - top2[0]))


@pytest.mark.slow
def test_xsharp_beam5(wmi, model_cache):
    """The one-clip beam launch at base (<512,5,beam>, per-row cross tasks
    with the cross q inside them) on base-xsharp's tone clip 1235, whose
    oracle search keeps every selection margin >= BEAM_GAP for 25 steps (the
    other seeds meet one within 1-8): every step's logits of every row and
    every selection against the oracle's search up to that step."""
    path = synth.model_path("base-xsharp", model_cache)
    om = pyoracle.OracleModel(path)
    try:
        _beam_step_logits_case(wmi, om, path, synth.synth_pcm_tones(30.0, 1235), 5, 40, 24, "base-xsharp 5 beams")
    finally:
        om.close()


def test_decoder_layernorm_large_mean_rows(wmi, model_cache):
    """The persistent decoder's one-pass LayerNorm statistics (E[x^2] -
    mean^2 in double; tests/test_ln_formula.py) on rows with |mean| / std up
    to ~700 (base-lnmean: decoder positional embedding + 16), against the
    oracle's two-pass ggml norm: every step's logits within the bar, on the
    one-row instance (ln1_vals) and on two clips (the multi-row ln_rows)."""
    path = synth.model_path("base-lnmean", model_cache)
    om = pyoracle.OracleModel(path)
    try:
        for n in (1, 2):
            clips = [synth.synth_pcm_tones(30.0, 1234 + i) for i in range(n)]
            _step_logits_case(wmi, om, path, clips, 32, tag=f"base-lnmean x{n}")
    finally:
        om.close()


def test_mel_dense_filterbank_layout_bitwise(micro_ctx, wmi, micro_model):
    """WMI_MEL_G=0: the mel layout a dense filterbank (more than MEL_FC_MAX
    non-zero weights) takes — 4 two-frame waves with the whole [201][n_mel]
    bank in LDS — gives bitwise the compact-bank layout's mel (same terms,
    same order)."""
    dense = _ctx_with_env(wmi, micro_model, {"WMI_MEL_G": "0"})
    try:
        for secs, seed in ((30.0, 7), (0.37, 3)):
            pcm = synth.synth_pcm_f32(secs, seed)
            outs = []
            for c in (micro_ctx, dense):
                c.pcm_to_mel_batch([pcm])
                outs.append(c.mel(0))
            np.testing.assert_array_equal(outs[0], outs[1])
    finally:
        dense.close()


# --- the multi-row and beam decoder instances at n > 512 (round-5 verdict
# item 1): every step's logits of every row against the oracle ---------------
@pytest.mark.slow
def test_step_logits_multi_row_small(wmi, model_cache):
    """<768,4>: small with four tone clips in one multi-row launch (MFMA
    GEMVs, multi-row LayerNorms, per-row cross tasks with the cross q inside
    them, MFMA logits above n = 512): every step's logits of every row
    within the bar against the oracle teacher-forced on that row's own ids."""
    path = synth.model_path("small", model_cache)
    om = pyoracle.OracleModel(path)
    try:
        clips = [synth.synth_pcm_tones(30.0, 1234 + i) for i in range(4)]
        _step_logits_case(wmi, om, path, clips, 32, tag="small x4 (<768,4>)", floor_clips=1)
    finally:
        om.close()


@pytest.mark.slow
def test_large_v3_xsharp_multi_row_ids_follow_the_audio(wmi, model_cache):
    """<1280,8>: large-v3-xsharp (synth.xsharp_lv3_hook: the audio drives the
    ids) on eight tone clips in one 8-row launch — the cross q from the D
    phase, per-row cross tasks, four waves splitting K in every MFMA GEMV and
    the logits: every step's logits of every row within the bar against the
    oracle teacher-forced on that row's ids, the ids = the oracle's argmax at
    every decisive step, and at least 6 distinct id sequences over the 8
    clips (a row / clip routing or cross K / V indexing bug changes a
    compared id or logit)."""
    path = synth.model_path("large-v3-xsharp", model_cache)
    om = pyoracle.OracleModel(path)
    try:
        clips = [synth.synth_pcm_tones(30.0, 1234 + i) for i in range(8)]
        got, dec = _step_logits_case(wmi, om, path, clips, 16, tag="large-v3-xsharp x8 (<1280,8>)", floor_clips=1)
        n_seq = len({tuple(x) for x in got})
        assert n_seq >= 6, n_seq
        assert min(dec) >= 12, dec
    finally:
        om.close()


def test_step_logits_beyond_one_block(wmi, micro_model, oracle_micro):
    """More clips than one 8-row block: each block's launch keeps
    its rows' logits at its own offset (rows 0-7: the split 8-row grid, rows
    8-9: a two-row launch), every row against the oracle."""
    clips = [synth.synth_pcm_tones(2.0, 500 + i) for i in range(10)]
    _step_logits_case(wmi, oracle_micro, micro_model, clips, 12, tag="micro x10 (two blocks)", n_ctx=64)


def _beam_step_logits_case(wmi, om, path, pcm, K, n_tok, min_steps, tag, n_ctx=1500, env=None):
    """C5's launch itself: a K-beam search with every step's logits kept
    (WMI_LOGITS_ALL: the beam launch's [K][V] rows each step) and the beam
    kernels' selections (parent slot, token per step), against the oracle's
    search with its per-step hypothesis logits (pyoracle decode_beam trace:
    the same dec_step as its teacher-forced decoder, so each row's logits are
    the oracle teacher-forced on that row's own history).  Every step while
    the two searches keep the same hypotheses, and the step where they part:
    each active row's logits within the bar; they may part only where the
    oracle's selection margin is below 2 x the bar (the logits' own noise),
    and not before min_steps.  The bar's floor is measured on the oracle's
    winning hypothesis.  Returns the steps with identical selections and the
    grid the beam launch ran on."""
    ctx = _ctx_with_env(wmi, path, dict(env or {}, WMI_LOGITS_ALL="1"))
    try:
        ctx.set_audio_ctx(n_ctx)
        ctx.pcm_to_mel_batch([pcm])
        ctx.encode(1, 0)
        got, got_score = ctx.decode_beam(K, n_tok, suppress_eot=True)[0]
        np_ = len(om.prompt())
        lg = ctx.step_logits(np_ + n_tok - 1)[np_ - 1:]
        dpar, dtok = ctx.beam_history(n_tok)
        grid = int(np.frombuffer(ctx.debug_read(17, 9 * 4), np.int32)[K])
    finally:
        ctx.close()
    kv = _oracle_encode(om, pcm, n_ctx)[1:]
    ref, score, gap, sg, tr = om.decode_beam(kv[0], kv[1], K, n_tok, suppress_eot=True, n_threads=threads(),
                                             step_gaps=True, trace=True)
    feed = np.array(list(om.prompt()) + list(ref[:-1]), np.int32)
    _, bar, floor = _logits_ref(om, kv, _exact_kv(om, pcm, n_ctx), feed)
    # the rows' histories (token tuples) on both sides: a device row is held
    # to the oracle hypothesis with the same history (two kept candidates
    # whose scores are closer than the f32 noise may take each other's slot)
    hd, ho = [()], [()]
    worst, rows, swaps, same = 0.0, 0, 0, n_tok
    for t in range(n_tok):
        where = {h: j for j, h in enumerate(ho)}
        for r, h in enumerate(hd):
            err = float(np.abs(lg[t, r] - tr["logits"][t, where[h]]).max())
            assert err <= bar, (tag, t, r, err, bar)
            worst, rows, swaps = max(worst, err), rows + 1, swaps + (where[h] != r)
        sel = tr["sel"][t]
        k = int((sel[:, 0] >= 0).sum())
        nd = [hd[int(p)] + (int(x),) for p, x in zip(dpar[t, :k], dtok[t, :k])]
        no = [ho[int(p)] + (int(x),) for p, x in sel[:k]]
        if set(nd) != set(no):
            # the searches part only where the oracle's selection margin is
            # within the logits' noise (2 x the bar) — a near-tie
            assert sg[t] < max(BEAM_GAP, 2 * bar), (tag, t, float(sg[t]), bar)
            same = t
            break
        hd, ho = nd, no
    print(f"[beam step logits] {tag}: grid {grid}; {min(same + 1, n_tok)} steps ({rows} hypothesis rows, "
          f"{swaps} in another slot than the oracle's) max |device - oracle| {worst:.3e} (bar {bar:.3e}, floor "
          f"{floor:.3e}); selections identical for {same} of {n_tok} steps"
          f"{'' if same == n_tok else f' (step {same}: oracle margin {sg[same]:.2e})'}; smallest oracle margin "
          f"before: {float(sg[:same].min()) if same else float('nan'):.2e}")
    assert same >= min_steps, (tag, same, sg[:same + 1])
    if same == n_tok:
        np.testing.assert_array_equal(got, ref)
        assert abs(got_score - score) < 2e-2, (got_score, score)
    return same, grid


@pytest.mark.slow
def test_beam_step_logits_large_v3_xsharp(wmi, model_cache):
    """C5's instance, <1280,5,beam> at 1500 frames with the beam rows sharing
    one cross task per (head, key chunk) (PersistArgs::xshare: 20 heads x 12
    chunks = 240 tasks within the grid), on an audio-dependent model
    (large-v3-xsharp, tone clip 1234: the oracle's 40 selection margins all
    >= BEAM_GAP, scripts/xsharp_probe.py): every step's logits of all five
    rows and every selection against the oracle over 40 steps, and the final
    hypothesis and score."""
    path = synth.model_path("large-v3-xsharp", model_cache)
    om = pyoracle.OracleModel(path)
    try:
        steps, grid = _beam_step_logits_case(wmi, om, path, synth.synth_pcm_tones(30.0, 1234), 5, 40, 32,
                                             "large-v3-xsharp 5 beams")
        assert grid >= 240, grid  # (the beam-shared cross tasks: H * ceil(T / 128) <= G)
    finally:
        om.close()


@pytest.mark.slow
def test_beam_small_grid_per_row_cross_tasks(wmi, model_cache, tmp_path):
    """The small-grid fallback of the beam launch (when
    H * ceil(T / 128) exceeds the grid the rows take per-row cross tasks
    instead of a rejected configuration): the library built for a
    192-workgroup grid (variants/g192, WMI_GDESIGN=192; 20 x 12 = 240 > 192)
    runs large-v3's 5-beam search in a child process and gives bitwise the
    tokens, score, selections and every step's logits of the default
    256-workgroup build with shared cross tasks — neither the grid nor the
    task layout enters a row's arithmetic (MFMA GEMVs in a fixed wave order,
    test_beam_shared_cross_equals_per_row)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib192 = os.path.join(root, "whisper.rs_amd", "variants", "g192", "libwhisper_mi355x.so")
    assert os.path.exists(lib192), "build the variants (make -C whisper.rs_amd/csrc)"
    path = synth.model_path("large-v3", model_cache)
    out = str(tmp_path / "g192.npz")
    env = dict(os.environ, WMI_LIB=lib192)
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "beam_worker.py"), path, "1236", "5", "12", out],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    small = np.load(out)
    ctx = _ctx_with_env(wmi, path, {"WMI_LOGITS_ALL": "1"})
    try:
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, 1236)])
        ctx.encode(1, 0)
        toks, score = ctx.decode_beam(5, 12, suppress_eot=True)[0]
        par, tok = ctx.beam_history(12)
        lg = ctx.step_logits(4 + 12 - 1)[3:, :5]
        grids = np.frombuffer(ctx.debug_read(17, 9 * 4), np.int32)
    finally:
        ctx.close()
    print(f"[small grid] beam grid: g192 build {int(small['grids'][5])}, default {int(grids[5])}")
    assert int(small["grids"][5]) == 192 and int(grids[5]) >= 240
    np.testing.assert_array_equal(small["tokens"], toks)
    assert float(small["score"]) == score
    np.testing.assert_array_equal(small["par"], par)
    np.testing.assert_array_equal(small["tok"], tok)
    np.testing.assert_array_equal(small["logits"], lg)
