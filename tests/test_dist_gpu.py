"""The RCCL data path on one GPU: a world-1 communicator through the C ABI.

bench.py --gpus N gathers every rank's token block to rank 0 with
wmi_dist_gather_tokens (ncclGather) and fences with wmi_dist_barrier
(ncclAllReduce).  With world = 1 the same calls run the same RCCL code on a
single device, so the block layout ([clips][1 + n_decode]: count, then the
tokens) and both decode modes are checked against wmi_get_tokens here; the
multi-rank sharding is covered on CPU (tests/test_dist_cpu.py).
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wmi():
    import wmi as w
    return w


def test_rccl_world1_gather_greedy_and_beam(wmi, micro_model):
    ctx = wmi.WhisperContext.new(micro_model, 0, max_clips=2)
    try:
        uid = wmi.WhisperContext.dist_make_id()
        assert len(uid) == wmi.lib().wmi_dist_id_size()
        ctx.dist_init(0, 1, uid)
        ctx.stage([synth.synth_pcm_f32(2.0, 11), synth.synth_pcm_f32(2.0, 12)])

        # greedy: the device token block, counts = n_decode (EOT suppressed)
        ctx.run_staged(n_decode=16)
        toks, counts = ctx.dist_gather_tokens()
        assert toks.shape == (1, 2, 16) and counts.shape == (1, 2)
        np.testing.assert_array_equal(toks[0], ctx.tokens())
        assert (counts == 16).all()
        ctx.dist_barrier()
        again, _ = ctx.dist_gather_tokens()  # the barrier touches no token buffer
        np.testing.assert_array_equal(again, toks)

        # beam: the best sequences live on the host; the block is padded with -1
        ctx.run_staged(n_decode=8, beam_size=2)
        btoks, bcounts = ctx.dist_gather_tokens()
        np.testing.assert_array_equal(btoks[0], ctx.tokens())
        ref = ctx.decode_beam(2, 8, suppress_eot=True)  # same encoded clips, same search
        for c, (seq, _) in enumerate(ref):
            assert bcounts[0, c] == len(seq)
            np.testing.assert_array_equal(btoks[0, c, :len(seq)], seq)
            assert (btoks[0, c, len(seq):] == -1).all()
        ctx.dist_barrier()
    finally:
        ctx.close()


def test_gather_before_run_is_an_error(wmi, micro_model):
    ctx = wmi.WhisperContext.new(micro_model, 0, max_clips=1)
    try:
        ctx.dist_init(0, 1, wmi.WhisperContext.dist_make_id())
        ctx._n_decode = 4
        with pytest.raises(wmi.InvalidArgument):
            ctx.dist_gather_tokens()
    finally:
        ctx.close()


def test_tuning_knobs_are_per_context(wmi, micro_model, monkeypatch):
    """WMI_* knobs are read into the context at init: a context created
    under one setting keeps it while another context, created on another
    thread under a different environment, gets its own."""
    import threading
    monkeypatch.setenv("WMI_LOGITS_CAP", "64")
    monkeypatch.setenv("WMI_GRAPH_STEPS", "4")
    a = wmi.WhisperContext.new(micro_model, 0, max_clips=1)
    monkeypatch.delenv("WMI_LOGITS_CAP")
    monkeypatch.delenv("WMI_GRAPH_STEPS")
    box = {}
    t = threading.Thread(target=lambda: box.update(b=wmi.WhisperContext.new(micro_model, 0, max_clips=1)))
    t.start()
    t.join(120)
    b = box["b"]
    try:
        ka = np.frombuffer(a.debug_read(10, 36), np.int32)
        kb = np.frombuffer(b.debug_read(10, 36), np.int32)
        assert ka[0] == 64 and ka[4] == 4    # logits_cap, graph_steps of the first context
        assert kb[0] == 512 and kb[4] == 8   # defaults in the second
        # and both run to the same numbers
        pcm = synth.synth_pcm_f32(2.0, 5)
        outs = []
        for c in (a, b):
            c.pcm_to_mel_batch([pcm])
            c.encode(1, 0)
            outs.append(c.encoder_out())
        np.testing.assert_allclose(outs[0], outs[1], atol=2e-3)
    finally:
        a.close()
        b.close()
