#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on the MI355X-native Whisper hot path.

One step = the whole hot path for one batch of synthetic 30 s clips already
resident in HBM: log-mel -> conv stem -> encoder -> ln_post -> cross-attention
K/V -> 128 greedy decoder tokens (EOT suppressed) per clip.
N = 1 is configs[1] (Whisper base f16, one 30 s clip, 1 x MI355X).  With
--gpus N the driver launches one process per GPU (torch.distributed.run env);
each rank owns --clips-per-gpu clips (weak scaling, configs[3] shards 8 clips
per GPU) and the token ids of every rank are gathered to rank 0 with RCCL
(ncclGather over xGMI) inside the timed step.  Rank 0 prints one JSON line.

value = audio seconds transcribed per wall second over all ranks (= 1/RTF
for one clip on one GPU); ms_per_step is the max over ranks.  The line also
carries the per-stage device times (encoder_ms etc.), the dominant kernel's
roofline (HIP events, live) and the CPU restatement timed on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "whisper.rs_amd"))

import dist  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense FP16
# wmi_bench_kernel ids timed live (HIP events on the context's stream).  14 is
# the persistent greedy decoder, the top kernel of the bench command's rocprof
# table (profiles/r02_bench_base_kernel_stats.csv: one launch per step, ~94%
# of GPU time); 1-3 are the top encoder kernels.
KERNELS = {14: ("hbm", "dec_persist"), 1: ("mfma", "enc_mlp0"), 2: ("mfma", "enc_attn"), 3: ("mfma", "cross_kv")}
# roofline.traffic: per-launch HBM-side bytes of the roofline kernel from
# rocprofv3 PMC counters over the same template instance and workload
# (scripts/pmc_pass.sh + scripts/pmc_summary.py; the profiler cannot run
# inside this process), keyed by (model, kernel id, n_decode)
PMC_TRAFFIC = {("base", 14, 128): "profiles/r02b_pmc_persist_base.json"}


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


def time_oracle(om, clip, n_decode: int, threads: int, min_seconds: float, max_seconds: float):
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
    sec, n, st = time_oracle(om, clip, n_decode, threads, min_seconds, max_seconds)
    sec1, n1, st1 = time_oracle(om, clip, n_decode, 1, 0.0, max_seconds)
    om.close()
    audio = len(clip) / synth.SAMPLE_RATE
    tiny = pyoracle.OracleModel(synth.model_path("tiny.en"))
    jfk = synth.synth_pcm_f32(11.0, 4321)
    tsec, tn, _ = time_oracle(tiny, jfk, n_decode, threads, min_seconds / 4, max_seconds / 2)
    tsec1, tn1, _ = time_oracle(tiny, jfk, n_decode, 1, 0.0, max_seconds / 2)
    tiny.close()
    return {
        "value": audio / sec,
        "unit": "audio-s/s",
        "cores": threads,
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


def whole_step_bytes(hp: dict, clips: int, dec_bytes: float) -> float:
    """Algorithmic bytes of one bench step: the decode launch's (wmi_bench_kernel
    14) plus the mel input, the encoder and cross-K/V weights and the encoder
    activations written once and read once per layer (f16)."""
    n, L, T, nm = hp["n_audio_state"], hp["n_audio_layer"], hp["n_audio_ctx"], hp["n_mels"]
    w = 2.0 * (3 * nm * n + 3 * n * n + L * 12 * n * n + hp["n_text_layer"] * 2 * hp["n_text_state"] * n)
    act = clips * (480000 * 4 + L * T * 56 * n)  # per layer and frame: x, LN, QKV, attention, MLP in and out
    return dec_bytes + w + act


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="base")
    ap.add_argument("--clips-per-gpu", type=int, default=1)
    ap.add_argument("--n-decode", type=int, default=128)
    ap.add_argument("--beam", type=int, default=0, help="beam width (0 = greedy; C5 uses 5)")
    ap.add_argument("--roofline-kernel", type=int, default=14, choices=sorted(KERNELS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-min-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-max-seconds", type=float, default=30.0)
    args = ap.parse_args()

    rank, world, local = dist.env_rank_world()
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using the launcher's world size")
    group = dist.Group(rank, world)
    cpg = args.clips_per_gpu
    path = synth.model_path(args.model)
    clips = [synth.synth_pcm_f32(30.0, sd) for sd in clip_seeds(rank, cpg)]
    audio_s = 30.0 * cpg

    import wmi
    ctx = wmi.WhisperContext.new(path, device=local, max_clips=cpg)
    if world > 1:
        uid = group.broadcast(wmi.WhisperContext.dist_make_id() if rank == 0 else None)
        ctx.dist_init(rank, world, uid)
    ctx.stage(clips)

    def step():
        ctx.run_staged(n_decode=args.n_decode, beam_size=args.beam)
        if world > 1:
            ctx.dist_gather_tokens()

    for i in range(args.warmup):
        step()
        log(f"warmup {i + 1}/{args.warmup}")
    if world > 1:
        ctx.dist_barrier()
    group.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    if world > 1:
        ctx.dist_barrier()
    t1 = time.perf_counter()
    group.barrier()
    elapsed = group.max(t1 - t0)
    tm = ctx.timings()
    log(f"timed {args.steps} steps in {elapsed * 1e3:.1f} ms; stage times {tm}")

    result = None
    if rank == 0:
        wtype = "q5_1" if args.model.endswith("q5_1") else "f16"
        ms_step = elapsed / args.steps * 1e3
        value = world * audio_s * args.steps / elapsed
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
        whole = {"alg_bytes": step_bytes, "ms": round(ms_step, 3),
                 "GB/s": round(step_bytes / (ms_step * 1e-3) / 1e9, 1),
                 "frac": round(step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        result = {
            "metric": "real-time factor + encoder ms, Whisper-base 30s audio, 1 GPU and 8-GPU batch",
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
                "parallelism": f"{world} replica(s), RCCL gather of token ids" if world > 1 else "1 GPU",
            },
            "rtf": round(ms_step / 1e3 / (audio_s), 6),
            "encoder_ms": round(tm["encode_ms"] + tm["cross_kv_ms"], 3),
            "stage_ms": {k: round(v, 3) if isinstance(v, float) else v for k, v in tm.items()},
            "roofline": roof,
            "whole_step": whole,
            "kernels": kernels,
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU restatement (bounded sample)")
        result["cpu_baseline"] = cpu_baseline(path, clips[0], args.n_decode, args.cpu_min_seconds,
                                              args.cpu_max_seconds)
    elif rank == 0:
        result["cpu_baseline"] = None
    ctx.close()
    group.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
