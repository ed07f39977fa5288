"""Diagnostics for the persistent decoder: persist vs chain tokens, oracle margins."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle")]
import synth  # noqa: E402
import wmi  # noqa: E402


def ctx_env(path, env, mc):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return wmi.WhisperContext.new(path, 0, max_clips=mc)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def toks(path, env, seeds, n=60):
    ctx = ctx_env(path, env, len(seeds))
    ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, s) for s in seeds])
    ctx.encode(1, 0)
    out = ctx.decode_greedy(n, suppress_eot=True)
    ctx.close()
    return out


mode = sys.argv[1] if len(sys.argv) > 1 else "all"
if mode in ("all", "trace"):
    # trace [model] [rows]: phase clocks of a greedy run (rows clips at once)
    model = sys.argv[2] if len(sys.argv) > 2 else "base"
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    path = synth.model_path(model)
    toks(path, {"WMI_PTRACE": "1"}, list(range(40, 40 + rows)), 130 if model != "large-v3" else 40)
if mode == "beamtrace":
    # beamtrace [model] [K] [n]: phase clocks of a beam search (one launch per
    # step; phase A includes the launch gap and the beam kernels)
    model = sys.argv[2] if len(sys.argv) > 2 else "large-v3"
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    ctx = ctx_env(synth.model_path(model), {"WMI_PTRACE": "1"}, 1)
    ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, 1234)])
    ctx.encode(1, 0)
    ctx.decode_beam(K, n, suppress_eot=True)
    ctx.close()
if mode in ("all", "rows"):
    path = synth.model_path("base")
    P, C = {"WMI_PERSIST": "1"}, {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"}
    for seeds in ([40, 41], [41], [41, 40]):
        a, b = toks(path, P, seeds), toks(path, C, seeds)
        for i, s in enumerate(seeds):
            print("seeds", seeds, "clip seed", s, "persist", a[i][8:13], "chain", b[i][8:13],
                  "diff at", np.nonzero(a[i] != b[i])[0][:4], flush=True)
    import pyoracle
    om = pyoracle.OracleModel(path)
    mel = om.mel(synth.synth_pcm_f32(30.0, 41), n_threads=16)
    _, ck, cv = om.encode(mel, n_ctx=1500, n_threads=16)
    ref, margins = om.decode_greedy(ck, cv, 14, suppress_eot=True, n_threads=16)
    print("oracle seed 41", ref[8:13], "margins", np.round(margins[8:13], 5), flush=True)

if mode == "logits":
    # last-step logits and final residual stream: persistent decoder vs chain (unfused)
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    hp = None
    res = {}
    for name, env in (("persist", {"WMI_PERSIST": "1", "WMI_PERSIST_LOGITS": "1"}),
                      ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})):
        ctx = ctx_env(path, env, 1)
        hp = ctx.hparams
        n, V = hp["n_text_state"], hp["n_vocab"]
        ctx.pcm_to_mel_batch(pcm)
        ctx.encode(1, 0)
        tk = ctx.decode_greedy(int(sys.argv[2]) if len(sys.argv) > 2 else 11, suppress_eot=True)[0]
        lg = np.frombuffer(ctx.debug_read(2, 8 * V * 4), np.float32)[:V]
        if name == "persist":
            xg = np.frombuffer(ctx.debug_read(3, 8 * 8 * n * 8), np.uint64)
            x = (xg[:n] & 0xffffffff).astype(np.uint32).view(np.float32)
        else:
            x = np.frombuffer(ctx.debug_read(0, 8 * n * 4), np.float32)[:n]
        res[name] = (tk, lg.copy(), x.copy())
        ctx.close()
    (tp, lp, xp), (tc, lc, xc) = res["persist"], res["chain"]
    print("tokens persist", tp, "\ntokens chain  ", tc)
    d = np.abs(lp - lc)
    print("logits max|d|", d.max(), "at", int(d.argmax()), "n differing", int((d > 0).sum()))
    for nm, l in (("persist", lp), ("chain", lc)):
        o = np.argsort(l)[-3:][::-1]
        print(nm, "top3", o, l[o])
    dx = np.abs(xp - xc)
    print("final x max|d|", dx.max(), "n differing", int((dx > 0).sum()), "of", len(dx))

if mode == "oracle":
    # teacher-forced oracle logits at the last step vs both decoders
    import pyoracle
    path = synth.model_path("base")
    pcm = synth.synth_pcm_f32(30.0, 41)
    om = pyoracle.OracleModel(path)
    mel = om.mel(pcm, n_threads=16)
    _, ck, cv = om.encode(mel, n_ctx=1500, n_threads=16)
    ngen = int(sys.argv[2])
    for name, env in (("persist", {"WMI_PERSIST": "1", "WMI_PERSIST_LOGITS": "1"}),
                      ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})):
        ctx = ctx_env(path, env, 1)
        V = ctx.hparams["n_vocab"]
        ctx.pcm_to_mel_batch([pcm])
        ctx.encode(1, 0)
        tk = ctx.decode_greedy(ngen, suppress_eot=True)[0]
        lg = np.frombuffer(ctx.debug_read(2, 8 * V * 4), np.float32)[:V].copy()
        feed = np.array(om.prompt() + list(tk[:ngen - 1]), np.int32)
        ref = om.decode_logits(ck, cv, feed, n_threads=16)[-1]
        d = np.abs(lg - ref)
        print(name, "last-step logits vs oracle: max", d.max(), "mean", d.mean(), flush=True)
        ctx.close()
    om.close()

if mode == "layers":
    # first (layers, n_gen) at which the two decoders' last-step logits differ
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    for L in range(1, 7):
        ctxs = []
        for env in ({"WMI_PERSIST": "1", "WMI_PERSIST_LOGITS": "1", "WMI_DEC_LAYERS": str(L)},
                    {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1", "WMI_DEC_LAYERS": str(L)}):
            c = ctx_env(path, env, 1)
            c.pcm_to_mel_batch(pcm)
            c.encode(1, 0)
            ctxs.append(c)
        V = ctxs[0].hparams["n_vocab"]
        first = None
        for n in range(1, 21):
            lg = []
            for c in ctxs:
                c.decode_greedy(n, suppress_eot=True)
                lg.append(np.frombuffer(c.debug_read(2, 8 * V * 4), np.float32)[:V].copy())
            d = np.abs(lg[0] - lg[1]).max()
            if d > 0:
                first = (n, d)
                break
        print("layers", L, "first differing n_gen", first, flush=True)
        for c in ctxs:
            c.close()

if mode == "state":
    # last-step layer-(L-1) state of both decoders: q, hidden, KV cache rows, final x
    L, ngen = int(sys.argv[2]), int(sys.argv[3])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    st = {}
    for name, env in (("persist", {"WMI_PERSIST": "1", "WMI_PERSIST_LOGITS": "1", "WMI_DEC_LAYERS": str(L)}),
                      ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1", "WMI_DEC_LAYERS": str(L)})):
        c = ctx_env(path, env, 1)
        hp = c.hparams
        n, V, Lt, tctx = hp["n_text_state"], hp["n_vocab"], hp["n_text_layer"], hp["n_text_ctx"]
        c.pcm_to_mel_batch(pcm)
        c.encode(1, 0)
        tk = c.decode_greedy(ngen, suppress_eot=True)[0]
        kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)
        vc = np.frombuffer(c.debug_read(7, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)
        lg = np.frombuffer(c.debug_read(2, 8 * V * 4), np.float32)[:V].copy()
        st[name] = (tk, kc.copy(), vc.copy(), lg)
        c.close()
    (tp, kp, vp, lp), (tcn, kcn, vcn, lc) = st["persist"], st["chain"]
    npos = 3 + ngen - 1
    print("tokens equal:", (tp == tcn).all(), "logits max|d|", np.abs(lp - lc).max())
    for l in range(L):
        for p_ in range(npos):
            dk = int((kp[l, 0, p_] != kcn[l, 0, p_]).sum())
            dv = int((vp[l, 0, p_] != vcn[l, 0, p_]).sum())
            if dk or dv:
                print(f"layer {l} pos {p_}: k differs in {dk}, v in {dv} of {n}", flush=True)
                break

if mode == "determinism":
    # KV caches of repeated runs: persistent x2, chain x2, chain eager
    L, ngen = int(sys.argv[2]), int(sys.argv[3])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    runs = {}
    for name, env in (("persist_a", {"WMI_PERSIST": "1"}), ("persist_b", {"WMI_PERSIST": "1"}),
                      ("chain_a", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"}),
                      ("chain_b", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"}),
                      ("chain_eager", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1", "WMI_NO_GRAPH": "1"})):
        env["WMI_DEC_LAYERS"] = str(L)
        c = ctx_env(path, env, 1)
        hp = c.hparams
        n, Lt, tctx = hp["n_text_state"], hp["n_text_layer"], hp["n_text_ctx"]
        c.pcm_to_mel_batch(pcm)
        c.encode(1, 0)
        c.decode_greedy(ngen, suppress_eot=True)
        kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)[:L, 0, :3 + ngen]
        runs[name] = kc.copy()
        c.close()
    names = list(runs)
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            d = np.argwhere(runs[names[i]] != runs[names[j]])
            print(names[i], "vs", names[j], "differing k elements", len(d), d[:3].tolist(), flush=True)
    a, b = runs["persist_a"], runs["chain_a"]
    for (l, p_, c_) in np.argwhere(a != b)[:4]:
        fa = np.array([a[l, p_, c_]], np.uint16).view(np.float16)[0]
        fb = np.array([b[l, p_, c_]], np.uint16).view(np.float16)[0]
        print("layer", l, "pos", p_, "col", c_, "persist", fa, "chain", fb)

if mode == "qkv":
    # this step's q / k / v of the last layer: persistent granules vs chain buffers
    L, ngen = int(sys.argv[2]), int(sys.argv[3])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    out = {}
    for name, env in (("persist", {"WMI_PERSIST": "1"}), ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})):
        env["WMI_DEC_LAYERS"] = str(L)
        c = ctx_env(path, env, 1)
        hp = c.hparams
        n, Lt, tctx, H = hp["n_text_state"], hp["n_text_layer"], hp["n_text_ctx"], hp["n_text_head"]
        c.pcm_to_mel_batch(pcm)
        c.encode(1, 0)
        tk = c.decode_greedy(ngen, suppress_eot=True)[0]
        kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)
        vc = np.frombuffer(c.debug_read(7, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)
        if name == "persist":
            xg = np.frombuffer(c.debug_read(3, 16 << 20), np.uint64)
            o_q = 3 * 8 * n  # persist_layout: x1, x2, x3 (8 n each), then q, k, v (4 n each)
            g = (xg & 0xffffffff).astype(np.uint32)
            q = g[o_q:o_q + n // 2].view(np.uint16)
            kk = g[o_q + 4 * n:o_q + 4 * n + n // 2].view(np.uint16)
            vv = g[o_q + 8 * n:o_q + 8 * n + n // 2].view(np.uint16)
            tags = (xg[o_q:o_q + n // 2] >> 32)
            print("persist q tags", np.unique(tags)[:4])
        else:
            q = np.frombuffer(c.debug_read(4, 8 * n * 2), np.uint16)[:n]
            kk = vv = None
        out[name] = (tk, q.copy(), kc[L - 1, 0].copy(), vc[L - 1, 0].copy(), None if kk is None else (kk.copy(), vv.copy()))
        c.close()
    tp, qp, kcp, vcp, (kk, vv) = out["persist"]
    tc, qc, kcc, vcc, _ = out["chain"]
    last = int(np.nonzero(kcc.any(axis=1))[0].max())
    print("tokens equal", (tp == tc).all(), "last written pos", last)
    print("q differs", int((qp != qc).sum()), "k(granules) vs persist cache", int((kk != kcp[last]).sum()),
          "v(granules) vs persist cache", int((vv != vcp[last]).sum()))
    print("k cache persist vs chain at last pos", int((kcp[last] != kcc[last]).sum()),
          "v", int((vcp[last] != vcc[last]).sum()))
    for p_ in range(last + 1):
        dk = np.nonzero(kcp[p_] != kcc[p_])[0]
        if len(dk):
            print("first pos with k diff", p_, "cols", dk[:8])
            break

if mode == "krow":
    # the cached k row of layer L-1, position P across run lengths, both decoders
    L, P, col = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    ctxs = {}
    for name, env in (("persist", {"WMI_PERSIST": "1"}), ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})):
        env["WMI_DEC_LAYERS"] = str(L)
        c = ctx_env(path, env, 1)
        c.pcm_to_mel_batch(pcm)
        c.encode(1, 0)
        ctxs[name] = c
    hp = ctxs["chain"].hparams
    n, Lt, tctx = hp["n_text_state"], hp["n_text_layer"], hp["n_text_ctx"]
    for ngen in range(P - 3 + 1, P - 3 + 9):
        row = {}
        for name, c in ctxs.items():
            c.decode_greedy(ngen, suppress_eot=True)
            kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)
            row[name] = kc[L - 1, 0, P].copy()
        d = np.nonzero(row["persist"] != row["chain"])[0]
        print("ngen", ngen, "last pos", 4 + ngen - 2, "k[P] diff cols", d[:6],
              "persist", row["persist"][col], "chain", row["chain"][col], flush=True)

if mode == "tf":
    # teacher-forced logits, both decoders, per position; first position that differs
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    rng = np.random.default_rng(3)
    for L in (1, 2, 6):
        res = []
        for env in ({"WMI_PERSIST": "1"}, {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"}):
            env["WMI_DEC_LAYERS"] = str(L)
            c = ctx_env(path, env, 1)
            c.pcm_to_mel_batch(pcm)
            c.encode(1, 0)
            toks = np.array([50258, 50259, 50359, 50363] + list(rng.integers(0, 50000, 60)), np.int32) if not res else res[0][0]
            lg = c.decode_logits(toks, 0)
            res.append((toks, lg))
            c.close()
        d = np.abs(res[0][1] - res[1][1]).max(axis=1)
        nz = np.nonzero(d)[0]
        print("layers", L, "positions", len(d), "first differing", nz[:5], "max", d.max(), flush=True)

if mode == "tfstate":
    # teacher-forced run of P + 1 tokens with L layers; last-step state of the last layer
    L, P = int(sys.argv[2]), int(sys.argv[3])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    rng = np.random.default_rng(3)
    toks = np.array([50258, 50259, 50359, 50363] + list(rng.integers(0, 50000, 60)), np.int32)[:P + 1]
    st = {}
    for name, env in (("persist", {"WMI_PERSIST": "1"}), ("chain", {"WMI_PERSIST": "0", "WMI_NO_FUSE": "1"})):
        env["WMI_DEC_LAYERS"] = str(L)
        c = ctx_env(path, env, 1)
        hp = c.hparams
        n, Lt, tctx, H, V = hp["n_text_state"], hp["n_text_layer"], hp["n_text_ctx"], hp["n_text_head"], hp["n_vocab"]
        T = 1500
        c.pcm_to_mel_batch(pcm)
        c.encode(1, 0)
        lg = c.decode_logits(toks, 0)[-1]
        kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)[L - 1, 0, P].copy()
        vc = np.frombuffer(c.debug_read(7, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)[L - 1, 0, P].copy()
        d = {"logits": lg, "k": kc, "v": vc}
        if name == "persist":
            g = (np.frombuffer(c.debug_read(3, 32 << 20), np.uint64) & 0xffffffff).astype(np.uint32)
            o = 0
            lay = {}
            for key, sz in (("x1", 8 * n), ("x2", 8 * n), ("x3", 8 * n), ("q", 4 * n), ("kg", 4 * n), ("vg", 4 * n),
                            ("o", 4 * n), ("xq", 4 * n), ("oc", 4 * n), ("h", 16 * n), ("s", 8 * H * T)):
                lay[key] = (o, sz)
                o += sz
            d["q"] = g[lay["q"][0]:lay["q"][0] + n // 2].view(np.uint16)
            d["x"] = g[lay["x1"][0]:lay["x1"][0] + n].view(np.float32)
            d["s"] = g[lay["s"][0]:lay["s"][0] + H * T].view(np.float32).reshape(H, T)
            d["h"] = g[lay["h"][0]:lay["h"][0] + 2 * n].view(np.uint16)
        else:
            d["q"] = np.frombuffer(c.debug_read(4, 8 * n * 2), np.uint16)[:n].copy()
            d["x"] = np.frombuffer(c.debug_read(0, 8 * n * 4), np.float32)[:n].copy()
            sst = np.frombuffer(c.debug_read(8, 8 * H * 1536 * 4), np.float32)
            d["s"] = sst[:H * 1536].reshape(H, 1536)[:, :T].copy()
            d["h"] = np.frombuffer(c.debug_read(5, 8 * 4 * n * 2), np.uint16)[:4 * n].copy()
        st[name] = d
        c.close()
    for key in ("q", "k", "v", "s", "h", "x", "logits"):
        a, b = st["persist"][key], st["chain"][key]
        dd = np.argwhere(a != b)
        print(f"{key:7s} differing {len(dd):6d} of {a.size}", dd[:4].tolist(), flush=True)

if mode == "selfattn":
    # layer-0 self-attention output at the last teacher-forced position P: persistent
    # decoder's o granules vs a float64 recomputation from the (shared) q / K / V
    P = int(sys.argv[2])
    path = synth.model_path("base")
    pcm = [synth.synth_pcm_f32(30.0, 41)]
    rng = np.random.default_rng(3)
    toks = np.array([50258, 50259, 50359, 50363] + list(rng.integers(0, 50000, 60)), np.int32)[:P + 1]
    c = ctx_env(path, {"WMI_PERSIST": "1", "WMI_DEC_LAYERS": "1"}, 1)
    hp = c.hparams
    n, Lt, tctx, H = hp["n_text_state"], hp["n_text_layer"], hp["n_text_ctx"], hp["n_text_head"]
    c.pcm_to_mel_batch(pcm)
    c.encode(1, 0)
    c.decode_logits(toks, 0)
    kc = np.frombuffer(c.debug_read(6, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)[0, 0, :P + 1].view(np.float16).astype(np.float64)
    vc = np.frombuffer(c.debug_read(7, Lt * 8 * tctx * n * 2), np.uint16).reshape(Lt, 8, tctx, n)[0, 0, :P + 1].view(np.float16).astype(np.float64)
    g = (np.frombuffer(c.debug_read(3, 32 << 20), np.uint64) & 0xffffffff).astype(np.uint32)
    q = g[3 * 8 * n:3 * 8 * n + n // 2].view(np.float16).astype(np.float64)
    o_g = g[3 * 8 * n + 12 * n:3 * 8 * n + 12 * n + n // 2].view(np.float16).astype(np.float64)
    c.close()
    worst = 0
    for h in range(H):
        s = kc[:, h * 64:(h + 1) * 64] @ q[h * 64:(h + 1) * 64]
        e = np.exp(np.float16(s - s.max()).astype(np.float64)).astype(np.float16).astype(np.float64)
        p16 = (e / e.sum()).astype(np.float32).astype(np.float16).astype(np.float64)
        o = p16 @ vc[:, h * 64:(h + 1) * 64]
        d = np.abs(o.astype(np.float16).astype(np.float64) - o_g[h * 64:(h + 1) * 64])
        ulp = np.spacing(np.abs(o).astype(np.float16)).astype(np.float64)
        worst = max(worst, (d / ulp).max())
        if (d / ulp).max() > 1:
            print("head", h, "max ulps", (d / ulp).max(), "at", int((d / ulp).argmax()))
    print("P", P, "self-attention o vs float64 recomputation: worst", worst, "f16 ulps", flush=True)
