"""Multi-process (world size 2) CPU test of the N > 1 path: bench.py's clip
sharding, the TCP rendezvous that carries the RCCL unique id / barrier /
max-over-ranks timing, and the gather of token ids — compared with gloo's
gather and with a single-process run over the whole batch.  The GPU data
path replaces the gather with ncclGather over xGMI (wmi_dist_gather_tokens)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shard_and_gather(micro_model):
    world, cpg, n_tok = 2, 2, 6
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), micro_model,
                                       str(cpg), str(n_tok)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    res = json.loads(outs[0][0].strip().splitlines()[-1])
    assert res["uid"] == "uid-from-rank0"
    assert res["tmax"] == 2.0
    tcp = np.array(res["tcp"])
    gloo = np.array(res["gloo"])
    assert tcp.shape == (world, cpg, n_tok)
    np.testing.assert_array_equal(tcp, gloo)
    # single process over the whole batch, clip c <- seed 1234 + c
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker
    full = np.concatenate([dist_worker.decode_shard(micro_model, r, cpg, n_tok) for r in range(world)])
    np.testing.assert_array_equal(tcp.reshape(world * cpg, n_tok), full)


def test_bench_launches_its_own_ranks():
    """`python3 bench.py --gpus 2` without torchrun's environment starts its two
    rank processes itself (configs[3]'s 8 clips per GPU by default), they meet
    over the TCP rendezvous, and rank 0's line carries n_gpus 2 and the max over
    ranks of the timed region (rank r sleeps (r + 1) * 10 ms per dry-run step)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["dry_run"] is True
    assert res["config"]["clips_per_gpu"] == 8 and res["config"]["global_clips"] == 16
    assert res["rendezvous"].startswith("tcp 127.0.0.1")
    assert len(res["rank_ms"]) == 2 and res["rank_ms"][1] >= 4 * 20.0
    assert abs(res["ms_per_step"] - max(res["rank_ms"]) / 4) < 1e-2
    assert abs(res["value"] / (2 * 8 * 30.0 * 4 / (max(res["rank_ms"]) / 1e3)) - 1) < 1e-3


def test_bench_launcher_fails_when_a_rank_fails():
    """A rank that exits non-zero makes the launcher exit non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--dry-run",
                        "--roofline-kernel", "99"], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0


def test_rendezvous_messages_are_data_only():
    """The TCP star carries JSON (bytes hex-tagged), never pickles."""
    import dist
    obj = [b"\x00\x01uid", 1.5, None, [1, 2, 3], "s"]
    assert dist._dec(dist._enc(obj)) == obj
    import pytest
    with pytest.raises(TypeError):
        dist._enc(object())
    with pytest.raises(ValueError):
        dist._dec(b'{"b": "00", "x": 1}')


def test_rendezvous_rejects_bad_ranks():
    """Rank 0 drops peers announcing an out-of-range or duplicate rank."""
    import struct
    import threading

    import dist
    port = _free_port()
    res = {}

    def hub():
        g = dist.Group(0, 2, "127.0.0.1", port, timeout=30)
        res["gather"] = g.all_gather("hub")
        g.close()

    t = threading.Thread(target=hub)
    t.start()
    import time
    for _ in range(100):  # the hub is listening once a connection succeeds
        try:
            rogue = socket.create_connection(("127.0.0.1", port), timeout=5)
            break
        except OSError:
            time.sleep(0.05)
    dist._send(rogue, struct.pack("<i", 7))  # world is 2: rank 7 is refused
    rogue.settimeout(5)
    assert rogue.recv(1) == b""  # closed by the hub
    rogue.close()
    peer = dist.Group(1, 2, "127.0.0.1", port, timeout=30)
    assert peer.all_gather("peer") == ["hub", "peer"]
    peer.close()
    t.join(30)
    assert res["gather"] == ["hub", "peer"]
