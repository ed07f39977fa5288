#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on the MI355X-native Whisper hot path.

One step = the whole hot path for one batch of synthetic 30 s clips already
resident in HBM: log-mel -> conv stem -> encoder -> ln_post -> cross-attention
K/V -> 128 greedy decoder tokens (EOT suppressed) per clip.
N = 1 is configs[1] (Whisper base f16, one 30 s clip, 1 x MI355X).

Multi-GPU (configs[3]: 64 clips, 8 per GPU): one process per GPU.  Launched by
torch.distributed.run, each rank reads RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* from the environment.  Launched as a plain `python3 bench.py --gpus N`
(no WORLD_SIZE), this process becomes a launcher: it starts the N rank
processes itself — before anything here touches a GPU — relays rank 0's JSON
line and exits non-zero if any rank fails.  Each rank owns --clips-per-gpu
clips (default 8 when N > 1: configs[3]'s shard; weak scaling) and the token
ids of every rank are gathered to rank 0 with RCCL (ncclGather over xGMI)
inside the timed step.

value = audio seconds transcribed per wall second over all ranks (= 1/RTF for
one clip on one GPU); ms_per_step is the max over ranks.  The N = 1 line also
carries the per-stage device times, the dominant kernel's roofline (HIP
events, live), every other single-GPU config of BASELINE.json measured in the
same run (`configs`), and the CPU restatement timed on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))

import dist  # noqa: E402
import synth  # noqa: E402

METRIC = "real-time factor + encoder ms, Whisper-base 30s audio, 1 GPU and 8-GPU batch"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense FP16
# wmi_bench_kernel ids timed live (HIP events on the context's stream).  14 is
# the persistent greedy decoder, the top kernel of the bench command's rocprof
# table (one launch per step, ~94% of GPU time); 1-3 are the top encoder kernels.
KERNELS = {14: ("hbm", "dec_persist"), 1: ("mfma", "enc_mlp0"), 2: ("mfma", "enc_attn"), 3: ("mfma", "cross_kv")}
# roofline.traffic: per-launch HBM-side bytes of the roofline kernel from
# rocprofv3 PMC counters over the same template instance and workload
# (scripts/pmc_pass.sh + scripts/pmc_summary.py; the profiler cannot run
# inside this process), keyed by (model, kernel id, n_decode)
PMC_TRAFFIC = {("base", 14, 128): "profiles/r06/final/pmc_persist_base.json"}
# the other single-GPU configs of BASELINE.json / north_star, measured in the
# same run as the headline (name -> model, clips, beam, steps, what it is)
EXTRA_CONFIGS = (
    ("tiny_f16", "tiny", 1, 0, 3, "north_star: tiny f16, one 30 s clip, 1 GPU"),
    ("small_f16", "small", 1, 0, 3, "north_star: small f16, one 30 s clip, 1 GPU"),
    ("c3_small_q5_1", "small-q5_1", 1, 0, 3, "configs[2]: small with ggml q5_1 weights, one 30 s clip, 1 GPU"),
    ("c4_shard_base_x8", "base", 8, 0, 3, "configs[3]'s per-GPU shard: base f16, 8 x 30 s clips on one GPU"),
    ("c5_large_v3_beam5", "large-v3", 1, 5, 2, "configs[4]: large-v3 f16, one 30 s clip, beam_size 5, 1 GPU"),
)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def clip_seeds(rank: int, clips_per_gpu: int):
    """Synthetic clip seeds of one rank: clip c of the global batch uses seed
    1234 + c; rank r owns clips [r * cpg, (r + 1) * cpg)."""
    return [1234 + rank * clips_per_gpu + i for i in range(clips_per_gpu)]


def cpu_model() -> str:
    """lscpu's 'Model name' (from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """CPUs this job may use: the OMP_NUM_THREADS share the GPU box grants a
    1-GPU job (16), else the process's affinity set (nproc)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def free_port() -> int:
    """A MASTER_PORT whose rendezvous hub ports (dist.hub_ports) can be bound
    too: checked by binding them, not assumed."""
    for _ in range(64):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p + dist.hub_ports(0)[-1] > 65535:
            continue
        try:
            t = socket.socket()
            t.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            t.bind(("127.0.0.1", dist.hub_ports(p)[0]))
            t.close()
            return p
        except OSError:
            t.close()
    raise OSError("no free rendezvous port")


def launch_ranks(n: int, argv, deadline_s: float) -> int:
    """Start one rank process of this script per GPU (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR, MASTER_PORT set as torch.distributed.run would),
    relay rank 0's result line and return non-zero if any rank fails: the
    first rank to exit non-zero (or by a signal) makes the launcher kill the
    others, and so does the deadline (deadline_s seconds for the whole run:
    a rank stuck in the rendezvous or in RCCL's init cannot hang the
    launcher).  Nothing in this process touches a GPU: it only imports the
    synthetic-input module (numpy) and generates the model file once, so the
    ranks do not race on it."""
    if "--dry-run" not in argv:
        model = "base"
        for i, a in enumerate(argv):
            if a == "--model" and i + 1 < len(argv):
                model = argv[i + 1]
            elif a.startswith("--model="):
                model = a.split("=", 1)[1]
        synth.model_path(model)
    port = free_port()
    log(f"launching {n} rank processes (rendezvous 127.0.0.1:{port}, deadline {deadline_s:.0f} s)")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []  # rank 0's stdout, drained while the ranks run (a full pipe would stall it)
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    t_end = time.monotonic() + deadline_s
    rc = 0
    while True:
        states = [p.poll() for p in procs]
        bad = [(r, s) for r, s in enumerate(states) if s not in (None, 0)]
        if bad:
            rc = bad[0][1]
            log(f"rank {bad[0][0]} exited with status {rc}; stopping the other ranks")
            break
        if all(s == 0 for s in states):
            break
        if time.monotonic() > t_end:
            log(f"deadline of {deadline_s:.0f} s passed with rank(s) "
                f"{[r for r, s in enumerate(states) if s is None]} still running; stopping every rank")
            rc = 124
            break
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.kill()
    for p in procs:
        p.wait()
    reader.join(10)
    lines = [ln for ln in (out[0] if out else b"").decode().splitlines() if ln.startswith("{")]
    if rc == 0 and lines:
        print(lines[-1], flush=True)
    elif rc == 0:
        log("rank 0 printed no result line")
        rc = 1
    return rc if rc > 0 else 1 if rc else 0


def cycle_oracle(om, clip, n_decode: int, threads: int, min_seconds: float, max_seconds: float):
    """Full clips (mel with main.rs:1698's 4 threads, encoder + cross K/V,
    n_decode greedy tokens) on the C restatement until min_seconds elapse;
    returns (seconds per clip, clips, per-stage seconds)."""
    n_ctx = om.hp["n_audio_ctx"]
    done, t_total, st = 0, 0.0, [0.0, 0.0, 0.0]
    while True:
        t0 = time.perf_counter()
        mel = om.mel(clip, n_threads=min(4, threads))
        t1 = time.perf_counter()
        _, ck, cv = om.encode(mel, n_ctx=n_ctx, n_threads=threads)
        t2 = time.perf_counter()
        om.decode_greedy(ck, cv, n_decode, suppress_eot=True, n_threads=threads)
        t3 = time.perf_counter()
        st = [st[0] + t1 - t0, st[1] + t2 - t1, st[2] + t3 - t2]
        done += 1
        t_total += t3 - t0
        if t_total >= min_seconds or t_total + (t3 - t0) > max_seconds:
            break
    return t_total / done, done, [x / done for x in st]


def cpu_baseline(model_path: str, clip, n_decode: int, min_seconds: float, max_seconds: float):
    """The C restatement (oracle/) on the host cores: the bench's own workload
    (base, one 30 s clip) with all granted threads and with one thread, plus
    configs[0] (tiny.en on an 11 s clip, the length of the reference README's
    jfk.wav, which the reference tree does not hold)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # test infrastructure; only this leg of bench.py loads it
    threads = cpu_threads()
    om = pyoracle.OracleModel(model_path)
    sec, n, st = cycle_oracle(om, clip, n_decode, threads, min_seconds, max_seconds)
    sec1, n1, st1 = cycle_oracle(om, clip, n_decode, 1, 0.0, max_seconds)
    om.close()
    audio = len(clip) / synth.SAMPLE_RATE
    tiny = pyoracle.OracleModel(synth.model_path("tiny.en"))
    jfk = synth.synth_pcm_f32(11.0, 4321)
    tsec, tn, _ = cycle_oracle(tiny, jfk, n_decode, threads, min_seconds / 4, max_seconds / 2)
    tsec1, tn1, _ = cycle_oracle(tiny, jfk, n_decode, 1, 0.0, max_seconds / 2)
    tiny.close()
    return {
        "value": audio / sec,
        "unit": "audio-s/s",
        "cores": threads,
        "cores_note": (f"{threads} = the CPU share (OMP_NUM_THREADS) the GPU box grants a 1-GPU job out of "
                       f"{os.cpu_count()} host CPUs; the 1-thread figure is t1_value (the C restatement's "
                       "threads split rows/heads, so time scales ~1/threads up to the memory-bandwidth limit)"),
        "kind": "port",
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "t1_value": audio / sec1,
        "sample": (f"{n} x full base clip at {threads} threads (mel {min(4, threads)} threads as main.rs:1698, "
                   f"encoder + cross K/V + {n_decode} greedy tokens): mel {st[0] * 1e3:.0f} ms, encoder "
                   f"{st[1] * 1e3:.0f} ms, decode {st[2] * 1e3:.0f} ms per clip; t1_value: {n1} clip at 1 thread "
                   f"(mel {st1[0] * 1e3:.0f}, encoder {st1[1] * 1e3:.0f}, decode {st1[2] * 1e3:.0f} ms); C "
                   "restatement of the reference (oracle/), not the reference binary (Rust, unbuildable here)"),
        "c1_tiny_en": {"value": 11.0 / tsec, "t1_value": 11.0 / tsec1, "unit": "audio-s/s", "cores": threads,
                       "sample": (f"configs[0]: tiny.en, 11 s synthetic clip (jfk.wav length), {n_decode} greedy "
                                  f"tokens; {tn} clip(s) at {threads} threads, {tn1} at 1 thread")},
    }


def encoder_flops(hp: dict) -> float:
    """Algorithmic encoder FLOP per 30 s clip: conv stem,
    per-layer QKV/O/MLP GEMMs, Q.K^T + P.V, cross K/V."""
    n, L, T, nm = hp["n_audio_state"], hp["n_audio_layer"], hp["n_audio_ctx"], hp["n_mels"]
    conv = 2.0 * 2 * T * n * 3 * nm + 2.0 * T * n * 3 * n
    layer = 2.0 * T * 4 * n * n + 2.0 * T * 8 * n * n + 4.0 * T * T * n
    return conv + L * layer + 2.0 * T * n * 2 * hp["n_text_layer"] * hp["n_text_state"]


def persist_q5(model: str) -> bool:
    """q5_1 files decode with the q5_1-block GEMVs unless WMI_PERSIST_Q5=0;
    beam launches read the f16 copies (wmi_persist.hip launch_ns)."""
    return model.endswith("q5_1") and os.environ.get("WMI_PERSIST_Q5", "1") != "0"


def decode_bytes(wmi, hp: dict, rows: int, steps: int, beam: bool, q5: bool) -> float:
    """Algorithmic bytes of one decode — the library's count
    (wmi_decode_alg_bytes, the one wmi_bench_kernel 14 reports): every step
    reads each decoder weight once (shared by the rows; the q5_1 GEMV matrices
    at their block size when the decode runs on them), the vocabulary matrix
    once, the cross K/V once per clip (beam rows share their clip's), and each
    row's self K/V rows [0, pos]; greedy rows run in blocks of 8."""
    return wmi.decode_alg_bytes(hp, rows, steps, beam, q5 and not beam)[0]


def measure_config(wmi, name, model, clips, beam, steps, warmup, n_decode, device, what):
    """One extra single-GPU config: its own context, staged clips, `steps`
    timed steps; stage times, the decoder's byte roofline and the encoder's
    MFMA fraction."""
    path = synth.model_path(model)
    ctx = wmi.WhisperContext.new(path, device=device, max_clips=clips)
    try:
        ctx.stage([synth.synth_pcm_f32(30.0, sd) for sd in clip_seeds(0, clips)])
        for _ in range(warmup):
            ctx.run_staged(n_decode=n_decode, beam_size=beam)
            ctx.tokens()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.run_staged(n_decode=n_decode, beam_size=beam)
            ctx.tokens()  # (ids on the host, as the headline step)
        el = time.perf_counter() - t0
        tm = ctx.timings()
        hp = ctx.hparams
        ms = el / steps * 1e3
        enc_ms = tm["encode_ms"] + tm["cross_kv_ms"]
        dec_steps = tm["n_decode_steps"]
        dbytes = decode_bytes(wmi, hp, clips if not beam else beam, dec_steps, bool(beam), persist_q5(model))
        dec = {"bound": "hbm", "alg_bytes": dbytes, "decode_ms": round(tm["decode_ms"], 3),
               "achieved": round(dbytes / (tm["decode_ms"] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        if not beam:
            try:  # the persistent decoder's own launch, timed live (HIP events); same byte count
                kb = ctx.bench_kernel(14, 1)
                dec.update(kernel=kb["name"], avg_us=round(kb["avg_us"], 1), alg_bytes=kb["alg_bytes"],
                           achieved=round(kb["alg_bytes"] / (kb["avg_us"] * 1e-6) / 1e9, 1))
            except Exception as e:  # the chain decoder ran (no persistent instance)
                log(f"{name}: kernel 14: {e}")
                dec["kernel"] = "decoder kernel chain"
        else:
            dec["kernel"] = f"k_dec_persist<{hp['n_text_state']},8,beam> per step + k_beam_topk/select"
        dec["frac"] = round(dec["achieved"] / HBM_PEAK_GBS, 4)
        ef = encoder_flops(hp) * clips
        return {
            "workload": what,
            "model": model,
            "clips": clips,
            "beam": beam,
            "steps": steps,
            "audio_s_per_s": round(30.0 * clips * steps / el, 2),
            "ms_per_step": round(ms, 3),
            "rtf": round(ms / 1e3 / (30.0 * clips), 6),
            "encoder_ms": round(enc_ms, 3),
            "mel_ms": round(tm["mel_ms"], 3),
            "decode_ms": round(tm["decode_ms"], 3),
            "decode_steps": dec_steps,
            "decode_us_per_step": round(tm["decode_ms"] * 1e3 / max(1, dec_steps), 1),
            "roofline": dec,
            "encoder_mfma": {"gflop": round(ef / 1e9, 2), "tflops": round(ef / (enc_ms * 1e-3) / 1e12, 1),
                             "frac": round(ef / (enc_ms * 1e-3) / 1e12 / MFMA_F16_PEAK_TFS, 4)},
        }
    finally:
        ctx.close()


def whole_step_bytes(hp: dict, clips: int, dec_bytes: float) -> float:
    """Algorithmic bytes of one bench step: the decode launch's (wmi_bench_kernel
    14) plus the mel input, the encoder and cross-K/V weights and the encoder
    activations written once and read once per layer (f16)."""
    n, L, T, nm = hp["n_audio_state"], hp["n_audio_layer"], hp["n_audio_ctx"], hp["n_mels"]
    w = 2.0 * (3 * nm * n + 3 * n * n + L * 12 * n * n + hp["n_text_layer"] * 2 * hp["n_text_state"] * n)
    act = clips * (480000 * 4 + L * T * 56 * n)  # per layer and frame: x, LN, QKV, attention, MLP in and out
    return dec_bytes + w + act


def run_rank(args, rank: int, world: int, local: int) -> None:
    group = dist.Group(rank, world)
    # test knobs (tests/test_dist_cpu.py): this rank fails, or hangs, right
    # after the rendezvous, so the launcher's kill / deadline paths run for real
    if os.environ.get("WMI_TEST_FAIL_RANK") == str(rank):
        log(f"rank {rank}: WMI_TEST_FAIL_RANK: exiting with status 3 after the rendezvous")
        sys.exit(3)
    if os.environ.get("WMI_TEST_HANG_RANK") == str(rank):
        log(f"rank {rank}: WMI_TEST_HANG_RANK: hanging after the rendezvous")
        time.sleep(3600)
    cpg = args.clips_per_gpu
    audio_s = 30.0 * cpg
    ctx = None
    if args.dry_run:
        # no device: the launcher, rendezvous and max-over-ranks timing only
        # (rank r "works" (r + 1) * 10 ms per step)
        def step():
            time.sleep(0.01 * (rank + 1))
    else:
        import wmi
        path = synth.model_path(args.model)
        clips = [synth.synth_pcm_f32(30.0, sd) for sd in clip_seeds(rank, cpg)]
        ctx = wmi.WhisperContext.new(path, device=local, max_clips=cpg)
        if world > 1:
            uid = group.broadcast(wmi.WhisperContext.dist_make_id() if rank == 0 else None)
            ctx.dist_init(rank, world, uid)
        ctx.stage(clips)

        def step():
            ctx.run_staged(n_decode=args.n_decode, beam_size=args.beam)
            if world > 1:
                ctx.dist_gather_tokens()  # every rank's ids to rank 0's host (ncclGather, then D2H)
            else:
                ctx.tokens()  # the ids the caller consumes, on the host (wmi_get_tokens: D2H)

    for i in range(args.warmup):
        step()
        log(f"rank {rank}: warmup {i + 1}/{args.warmup}")
    if ctx is not None and world > 1:
        ctx.dist_barrier()
    group.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    if ctx is not None and world > 1:
        ctx.dist_barrier()
    t1 = time.perf_counter()
    group.barrier()
    rank_s = group.all_gather(t1 - t0)
    elapsed = max(rank_s)
    log(f"rank {rank}: timed {args.steps} steps in {(t1 - t0) * 1e3:.1f} ms (max over ranks {elapsed * 1e3:.1f})")
    if rank != 0:
        if ctx is not None:
            ctx.close()
        group.close()
        return

    wtype = "q5_1" if args.model.endswith("q5_1") else "f16"
    ms_step = elapsed / args.steps * 1e3
    value = world * audio_s * args.steps / elapsed
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "audio-s/s (x real-time; 1/RTF)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic",
        "config": {
            "workload": (f"whisper-{args.model} {wtype} (random-init ggml-v1 weights), {cpg} x 30 s synthetic clip(s) "
                         f"per GPU: mel + conv stem + encoder + cross-KV + {args.n_decode} "
                         + (f"tokens of {args.beam}-beam search" if args.beam else "greedy tokens")),
            "beam": args.beam,
            "clips_per_gpu": cpg,
            "global_clips": world * cpg,
            "n_decode": args.n_decode,
            "parallelism": (f"{world} replicas (one process per GPU), RCCL gather of token ids" if world > 1
                            else "1 GPU"),
            "input": ("PCM staged in HBM before the timed region (wmi_stage_pcm; ~1.9 MB H2D per clip excluded, "
                      "about 0.03 ms at PCIe Gen5 rates); every step ends with the token ids on the host "
                      "(world 1: wmi_get_tokens; world > 1: the RCCL gather to rank 0)"),
        },
        "rank_ms": [round(s * 1e3, 3) for s in rank_s],
        "rendezvous": f"tcp {os.environ.get('MASTER_ADDR', '127.0.0.1')}" if world > 1 else None,
    }
    if args.dry_run:
        result["dry_run"] = True
        result["cpu_baseline"] = None
        group.close()
        print(json.dumps(result), flush=True)
        return

    tm = ctx.timings()
    kernels, kb_alg = {}, {}
    for k, (bound, name) in KERNELS.items():
        try:
            kb = ctx.bench_kernel(k, 3 if k == 14 else 50)
        except Exception as e:  # e.g. the persistent decoder not eligible for this shape
            log(f"kernel {name}: {e}")
            continue
        kb_alg[name] = kb["alg_bytes"]
        secs = kb["avg_us"] * 1e-6
        kernels[name] = {"kernel": kb["name"], "avg_us": round(kb["avg_us"], 3),
                         "GB/s": round(kb["alg_bytes"] / secs / 1e9, 1),
                         "TFLOP/s": round(kb["alg_flops"] / secs / 1e12, 2)}
    bound, name = KERNELS[args.roofline_kernel]
    roof = None
    if name in kernels:
        kd = kernels[name]
        if bound == "hbm":
            roof = {"bound": "hbm", "achieved": kd["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        else:
            roof = {"bound": "mfma", "achieved": kd["TFLOP/s"], "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof["traffic"] = None
        pmc = PMC_TRAFFIC.get((args.model, args.roofline_kernel, args.n_decode))
        if pmc and cpg == 1 and os.path.exists(os.path.join(ROOT, pmc)):
            with open(os.path.join(ROOT, pmc)) as fh:
                pm = json.load(fh)
            roof["traffic"] = pm["traffic_bytes"]  # HBM-side bytes per launch, rocprofv3 PMC (corrected)
            roof["traffic_source"] = pmc
        roof["alg_bytes"] = kb_alg[name]
        roof["kernel"] = kd["kernel"]
        roof["avg_us"] = kd["avg_us"]
    step_bytes = whole_step_bytes(ctx.hparams, cpg, kb_alg.get("dec_persist", 0.0))
    enc_ms = tm["encode_ms"] + tm["cross_kv_ms"]
    ef = encoder_flops(ctx.hparams) * cpg
    result.update({
        "rtf": round(ms_step / 1e3 / audio_s, 6),
        "encoder_ms": round(enc_ms, 3),
        "stage_ms": {k: round(v, 3) if isinstance(v, float) else v for k, v in tm.items()},
        "roofline": roof,
        "encoder_mfma": {"gflop": round(ef / 1e9, 2), "tflops": round(ef / (enc_ms * 1e-3) / 1e12, 1),
                         "frac": round(ef / (enc_ms * 1e-3) / 1e12 / MFMA_F16_PEAK_TFS, 4)},
        "whole_step": {"alg_bytes": step_bytes, "ms": round(ms_step, 3),
                       "GB/s": round(step_bytes / (ms_step * 1e-3) / 1e9, 1),
                       "frac": round(step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels": kernels,
    })
    ctx.close()
    ctx = None
    headline = world == 1 and args.model == "base" and cpg == 1 and args.beam == 0
    if world == 1 and (args.configs == "all" or (args.configs == "auto" and headline)):
        import wmi
        configs = {}
        for cname, model, clips, beam, steps, what in EXTRA_CONFIGS:
            log(f"config {cname}: {what}")
            try:
                configs[cname] = measure_config(wmi, cname, model, clips, beam, steps, 1, args.n_decode, local, what)
            except Exception as e:
                log(f"config {cname} failed: {e}")
                configs[cname] = {"workload": what, "error": str(e)}
        result["configs"] = configs
    if world == 1 and not args.no_cpu_baseline:
        log("timing the CPU restatement (bounded sample)")
        result["cpu_baseline"] = cpu_baseline(synth.model_path(args.model), synth.synth_pcm_f32(30.0, 1234),
                                              args.n_decode, args.cpu_min_seconds, args.cpu_max_seconds)
    else:
        result["cpu_baseline"] = None
    group.close()
    print(json.dumps(result), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="base")
    ap.add_argument("--clips-per-gpu", type=int, default=None,
                    help="clips per rank (default 1 at one GPU, 8 with --gpus > 1: configs[3]'s 64 = 8 x 8)")
    ap.add_argument("--n-decode", type=int, default=128)
    ap.add_argument("--beam", type=int, default=0, help="beam width (0 = greedy; C5 uses 5)")
    ap.add_argument("--roofline-kernel", type=int, default=14, choices=sorted(KERNELS))
    ap.add_argument("--configs", default="auto", choices=("auto", "all", "none"),
                    help="also measure BASELINE.json's other single-GPU configs (auto: with the headline run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-min-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-max-seconds", type=float, default=30.0)
    ap.add_argument("--launch-deadline", type=float, default=1500.0,
                    help="--gpus N without torchrun: seconds before the launcher kills every rank and fails")
    ap.add_argument("--dry-run", action="store_true",
                    help="no device: exercise the rank launcher, rendezvous and max-over-ranks timing on the CPU")
    args = ap.parse_args()
    if args.clips_per_gpu is None:
        args.clips_per_gpu = 8 if args.gpus > 1 else 1
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_deadline))
    rank, world, local = dist.env_rank_world()
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using the launcher's world size")
    run_rank(args, rank, world, local)


if __name__ == "__main__":
    main()
