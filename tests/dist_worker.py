"""Worker for tests/test_dist_cpu.py (not collected by pytest): one rank of a
CPU world that shards clips exactly as bench.py does, decodes them with the
oracle (micro model), and gathers token ids to rank 0 — once through the
repo's TCP rendezvous (whisper.rs_amd/dist.py) and once through
torch.distributed's gloo backend."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
import dist  # noqa: E402
import pyoracle  # noqa: E402
import synth  # noqa: E402


def decode_shard(model_path, rank, cpg, n_tok):
    om = pyoracle.OracleModel(model_path)
    out = []
    for sd in bench.clip_seeds(rank, cpg):
        mel = om.mel(synth.synth_pcm_f32(2.0, sd), n_threads=1)
        _, ck, cv = om.encode(mel, n_ctx=64, n_threads=1)
        out.append(om.decode_greedy(ck, cv, n_tok, suppress_eot=True, n_threads=1)[0])
    return np.stack(out).astype(np.int32)


def main():
    rank, world, _ = dist.env_rank_world()
    model_path, cpg, n_tok = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    g = dist.Group(rank, world)
    uid = g.broadcast(b"uid-from-rank0" if rank == 0 else None)
    toks = decode_shard(model_path, rank, cpg, n_tok)
    gathered = g.all_gather(toks.tolist())
    tmax = g.max(float(rank + 1))
    g.barrier()
    import torch
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.from_numpy(toks)
    bucket = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
    tdist.gather(t, bucket, dst=0)
    tdist.barrier()
    if rank == 0:
        print(json.dumps({"uid": uid.decode(), "tcp": gathered, "gloo": [b.tolist() for b in bucket], "tmax": tmax}))
    tdist.destroy_process_group()
    g.close()


if __name__ == "__main__":
    main()
