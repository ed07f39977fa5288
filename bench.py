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
KERNELS = {0: ("hbm", "dec_logits"), 1: ("mfma", "enc_mlp0"), 2: ("mfma", "enc_attn"), 3: ("mfma", "cross_kv"),
           4: ("hbm", "probe_empty"), 5: ("hbm", "probe_copy_1MiB")}
# roofline.traffic: per-launch HBM bytes of the roofline kernel measured with
# rocprofv3 PMC counters (scripts/pmc_pass.sh + scripts/pmc_summary.py; the
# profiler cannot run inside this process), keyed by (model, kernel id)
PMC_TRAFFIC = {("base", 0): "profiles/r01_pmc_logits_base.json"}


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def clip_seeds(rank: int, clips_per_gpu: int):
    """Synthetic clip seeds of one rank: clip c of the global batch uses seed
    1234 + c; rank r owns clips [r * cpg, (r + 1) * cpg)."""
    return [1234 + rank * clips_per_gpu + i for i in range(clips_per_gpu)]


def cpu_baseline(model_path: str, clip, n_decode: int, min_seconds: float, max_seconds: float):
    """The C restatement (oracle/) on the host cores: full pipeline per clip."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # test infrastructure; only this leg of bench.py loads it
    threads = min(16, os.cpu_count() or 8)
    om = pyoracle.OracleModel(model_path)
    n_ctx = om.hp["n_audio_ctx"]
    done, t_total, per_clip = 0, 0.0, []
    while True:
        t0 = time.perf_counter()
        mel = om.mel(clip, n_threads=4)  # main.rs:1698 hard-codes 4 mel threads
        t1 = time.perf_counter()
        _, ck, cv = om.encode(mel, n_ctx=n_ctx, n_threads=threads)
        t2 = time.perf_counter()
        om.decode_greedy(ck, cv, n_decode, suppress_eot=True, n_threads=threads)
        t3 = time.perf_counter()
        per_clip.append((t1 - t0, t2 - t1, t3 - t2))
        done += 1
        t_total += t3 - t0
        if t_total >= min_seconds or t_total + (t3 - t0) > max_seconds:
            break
    om.close()
    sec = t_total / done
    mel_s = sum(p[0] for p in per_clip) / done
    enc_s = sum(p[1] for p in per_clip) / done
    dec_s = sum(p[2] for p in per_clip) / done
    return {
        "value": 30.0 / sec,
        "unit": "audio-s/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{done} x full clip (mel 4 threads + encoder/cross-KV + {n_decode} greedy tokens, "
                   f"{threads} threads): mel {mel_s * 1e3:.0f} ms, encoder {enc_s * 1e3:.0f} ms, "
                   f"decode {dec_s * 1e3:.0f} ms per clip; C restatement of the reference (oracle/), "
                   "not the reference binary (unbuildable here)"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="base")
    ap.add_argument("--clips-per-gpu", type=int, default=1)
    ap.add_argument("--n-decode", type=int, default=128)
    ap.add_argument("--beam", type=int, default=0, help="beam width (0 = greedy; C5 uses 5)")
    ap.add_argument("--roofline-kernel", type=int, default=0, choices=sorted(KERNELS))
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
        kernels, kb_alg_bytes = {}, {}
        for k, (bound, name) in KERNELS.items():
            kb = ctx.bench_kernel(k, 50)
            kb_alg_bytes[name] = kb["alg_bytes"]
            secs = kb["avg_us"] * 1e-6
            kernels[name] = {"kernel": kb["name"], "avg_us": round(kb["avg_us"], 3),
                             "GB/s": round(kb["alg_bytes"] / secs / 1e9, 1),
                             "TFLOP/s": round(kb["alg_flops"] / secs / 1e12, 2)}
        bound, name = KERNELS[args.roofline_kernel]
        kd = kernels[name]
        if bound == "hbm":
            roof = {"bound": "hbm", "achieved": kd["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        else:
            roof = {"bound": "mfma", "achieved": kd["TFLOP/s"], "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof["traffic"] = None
        pmc = PMC_TRAFFIC.get((args.model, args.roofline_kernel))
        if pmc and os.path.exists(os.path.join(ROOT, pmc)):
            with open(os.path.join(ROOT, pmc)) as fh:
                pm = json.load(fh)
            roof["traffic"] = pm["traffic_bytes"]  # HBM bytes per launch, rocprofv3 PMC (corrected)
            roof["traffic_source"] = pmc
            roof["alg_bytes"] = kb_alg_bytes[name]
        roof["kernel"] = kd["kernel"]
        roof["avg_us"] = kd["avg_us"]
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
